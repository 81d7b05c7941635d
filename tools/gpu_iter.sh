#!/bin/bash
# One build→measure iteration on the GPU box: -m gpu tests (all, or -k expr), a kernel trace of
# selected kbench ops, and the default bench line without the CPU leg.
#   bash tools/gpu_iter.sh TAG "pytest -k expr | all" op1,op2,...
set -eo pipefail
TAG=$1; KEXPR=$2; OPS=$3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
if [ "$KEXPR" = "all" ]; then
  step tests 900 python -u -m pytest tests -m gpu -q -x --tb=short --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
else
  step tests 900 python -u -m pytest tests -m gpu -q -x --tb=short --timeout 300 --timeout-method thread -k "$KEXPR" > "$O/pytest.log" 2>&1
fi
tail -4 "$O/pytest.log"
grep -q " passed" "$O/pytest.log" && ! grep -q " failed" "$O/pytest.log" || { echo "tests failed"; exit 1; }
if [ -n "$OPS" ]; then
  step kbench 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 tools/kbench.py --ops "$OPS" --reps 20 --precision bf16x3 > "$O/kbench.log" 2>&1
  python3 - "$O/kt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r['Name'].startswith('void at::') or 'rocclr' in r['Name']:
        continue
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
fi
step bench 600 python3 bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
python3 -c "import json,sys; d=json.load(open('$O/bench.json')); print('BENCH', d['value'], d['ms_per_step'], d['alt_precisions'])"
