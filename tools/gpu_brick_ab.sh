#!/bin/bash
# Brick tile A/B (MRAGAN_BRICK_X3 = 0 default, 1 = 64x128 on 4 waves, 2 = 128x128 on 4 waves,
# 3 = 128x64 on 4 waves): bf16x3 brick parity tests and a kernel trace of res_fwd / res_dgrad each.
#   bash tools/gpu_brick_ab.sh TAG "0 1 2 3"
set -eo pipefail
TAG=$1; VARS=${2:-"0 1 2 3"}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
for v in $VARS; do
  export MRAGAN_BRICK_X3=$v
  step "tests v$v" 600 python -u -m pytest tests/test_kernels_gpu.py -q -x --tb=short --timeout 120 --timeout-method thread -k "bf16x3_fwd_dgrad or brick_presplit or conv_precision" > "$O/pytest_v$v.log" 2>&1
  tail -2 "$O/pytest_v$v.log"
  grep -q " failed" "$O/pytest_v$v.log" && { echo "v$v tests failed"; exit 1; }
  step "kbench v$v" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_v$v" -o run -- python3 tools/kbench.py --ops res_fwd,res_dgrad --reps 20 --precision bf16x3 > "$O/kbench_v$v.log" 2>&1
  python3 - "$O/kt_v$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'conv_brick' in r['Name']:
        print(f"v{sys.argv[2]} {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
