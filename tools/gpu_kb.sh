#!/bin/bash
# selected GPU tests + a kernel-trace of tools/kbench.py ops:
#   bash tools/gpu_kb.sh TAG "pytest -k expr" op1,op2,... [precision]
set -eo pipefail
TAG=$1; KEXPR=$2; OPS=$3; PREC=${4:-bf16x3}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
if [ -n "$KEXPR" ]; then
  step tests 900 python -u -m pytest tests -m gpu -q --tb=short --timeout 300 --timeout-method thread -k "$KEXPR" > "$O/pytest.log" 2>&1
  tail -4 "$O/pytest.log"
fi
step kbench 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 tools/kbench.py --ops "$OPS" --reps 20 --precision "$PREC" > "$O/kbench.log" 2>&1
python3 - "$O/kt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r['Name'].startswith('void at::') or 'rocclr' in r['Name']:
        continue
    print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
