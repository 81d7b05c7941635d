#!/bin/bash
# Brick tile sweep in one precision: for each "CFG/VAR" (MRAGAN_BRICK_CFG = "bm,bn" or "-" for the
# free choice, MRAGAN_BRICK_VAR = template variant of the 128x128 tile), the brick parity tests and a
# kernel trace of res_fwd / res_dgrad at N = 4 and N = 2 (64^3 b2 res-block shapes).
#   bash tools/gpu_brick_sweep.sh TAG PREC "-/0 128,128/0 128,128/1 128,128/2"
set -eo pipefail
TAG=$1; PREC=${2:-bf16}; VARS=${3:-"-/0"}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
i=0
for v in $VARS; do
  i=$((i + 1))
  cfg=${v%/*}; var=${v#*/}
  if [ "$cfg" = "-" ]; then unset MRAGAN_BRICK_CFG; else export MRAGAN_BRICK_CFG=$cfg; fi
  export MRAGAN_BRICK_VAR=$var
  step "tests $v" 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --tb=short --timeout 120 --timeout-method thread \
      -k "bf16x3_fwd_dgrad or brick_presplit or brick_in_stats" > "$O/pytest_$i.log" 2>&1
  tail -1 "$O/pytest_$i.log"
  grep -q " failed" "$O/pytest_$i.log" && { echo "$v tests failed"; exit 1; }
  for N in 4 2; do
    step "kbench $v N$N" 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${i}_$N" -o run -- \
        python3 tools/kbench.py --ops res_fwd,res_dgrad --reps 20 --precision "$PREC" --N $N > "$O/kbench_${i}_$N.log" 2>&1
    python3 - "$O/kt_${i}_$N" "$v N=$N" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'conv_brick' in r['Name'] or 'igemm' in r['Name']:
        print(f"{sys.argv[2]:>20s} {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
  done
done
echo "[sweep] done"
