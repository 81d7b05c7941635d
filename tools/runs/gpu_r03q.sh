#!/bin/bash
# r03q: brick tile variants whose waves share no weight fragment (MRAGAN_BRICK_VAR 3 / 4 / 1):
# parity under each variant, kernel A/B, step A/B.
set -eo pipefail
TAG=${1:-r03q}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
K="brick or op16"
step kt0 300 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread -k "$K" > "$O/kt0.log" 2>&1
tail -1 "$O/kt0.log"
step kt3 300 env MRAGAN_BRICK_VAR=3 MRAGAN_BRICK_CFG=64,128 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread -k "$K" > "$O/kt3.log" 2>&1
tail -1 "$O/kt3.log"
step kt4 300 env MRAGAN_BRICK_VAR=4 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread -k "$K" > "$O/kt4.log" 2>&1
tail -1 "$O/kt4.log"
step kt1 300 env MRAGAN_BRICK_VAR=1 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread -k "$K" > "$O/kt1.log" 2>&1
tail -1 "$O/kt1.log"
grep -h -E "^FAILED" "$O"/kt*.log | head || true
SETS="- MRAGAN_BRICK_VAR=1 MRAGAN_BRICK_VAR=4 MRAGAN_BRICK_CFG=64,128 MRAGAN_BRICK_VAR=3;MRAGAN_BRICK_CFG=64,128"
bash tools/gpu_ab_env.sh "$TAG/k4" bf16 4 res_fwd16,res_dgrad16 "$SETS"
bash tools/gpu_ab_env.sh "$TAG/k2" bf16 2 res_fwd16,res_dgrad16 "$SETS"
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- MRAGAN_BRICK_VAR=1 MRAGAN_BRICK_VAR=4 MRAGAN_BRICK_VAR=3;MRAGAN_BRICK_CFG=64,128 -"
echo "[r03q] done"
