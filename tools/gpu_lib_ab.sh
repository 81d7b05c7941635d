#!/bin/bash
# Same-box A/B of two library builds on kbench ops (kernel trace each):
#   B = mra-gan_amd/lib/ab/libmragan_hip.so (baseline), A = the in-tree build.
#   bash tools/gpu_lib_ab.sh TAG op1,op2 ["pytest -k expr"]
set -eo pipefail
TAG=$1; OPS=$2; KEXPR=${3:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
if [ -n "$KEXPR" ]; then
  step tests 900 python -u -m pytest tests -m gpu -q -x --tb=short --timeout 300 --timeout-method thread -k "$KEXPR" > "$O/pytest.log" 2>&1
  tail -2 "$O/pytest.log"
  grep -q " failed" "$O/pytest.log" && { echo "tests failed"; exit 1; }
fi
for side in base new; do
  if [ $side = base ]; then export MRAGAN_HIP_LIB=$R/mra-gan_amd/lib/ab/libmragan_hip.so; else unset MRAGAN_HIP_LIB; fi
  step "kbench $side" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$side" -o run -- python3 tools/kbench.py --ops "$OPS" --reps 20 --precision bf16x3 ${KB_ARGS:-} > "$O/kbench_$side.log" 2>&1
  python3 - "$O/kt_$side" "$side" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r['Name'].startswith('void at::') or 'rocclr' in r['Name']:
        continue
    print(f"{sys.argv[2]:4s} {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
