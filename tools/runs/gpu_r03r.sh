#!/bin/bash
# r03r: one-wave-per-SIMD brick tiles as the one-plane default; A/B against the 8-wave tiles (VAR=5)
set -eo pipefail
TAG=${1:-r03r}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "brick or op16 or step" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head || true
SETS="- MRAGAN_BRICK_VAR=5 MRAGAN_BRICK_CFG=64,128 MRAGAN_BRICK_CFG=128,64"
bash tools/gpu_ab_env.sh "$TAG/k4" bf16 4 res_fwd16,res_dgrad16 "$SETS"
bash tools/gpu_ab_env.sh "$TAG/k2" bf16 2 res_fwd16,res_dgrad16 "$SETS"
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- MRAGAN_BRICK_VAR=5 - MRAGAN_BRICK_VAR=5"
echo "[r03r] done"
