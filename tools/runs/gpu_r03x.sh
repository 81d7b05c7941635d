#!/bin/bash
# r03x: brickT conflict-free halo rows (104-row planes + lane table) vs HEAD (lib/ab/base)
set -eo pipefail
TAG=${1:-r03x}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "x3 or brickT or convT or in_stats or step" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head || true
B=MRAGAN_HIP_LIB=mra-gan_amd/lib/ab/base/libmragan_hip.so
bash tools/gpu_ab_env.sh "$TAG/k4" bf16 4 up2_fwd "- $B"
bash tools/gpu_ab_env.sh "$TAG/k2" bf16 2 up2_fwd "- $B"
bash tools/gpu_ab_env.sh "$TAG/x4" bf16x3 4 up2_fwd "- $B"
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- $B - $B"
echo "[r03x] done"
