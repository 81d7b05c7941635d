#!/bin/bash
# r03u: implicit GEMM without lo planes in the one-plane modes (LDS halved) vs the two-plane
# build (lib/ab/base, -DMRAGAN_IG_TWO_PLANES): parity + kernel A/B + step A/B
set -eo pipefail
TAG=${1:-r03u}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "x3 or igemm or in_stats or conv" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head || true
B=MRAGAN_HIP_LIB=mra-gan_amd/lib/ab/base/libmragan_hip.so
bash tools/gpu_ab_env.sh "$TAG/k4" bf16 4 down1_fwd,down2_fwd,up1_fwd,d2_fwd "- $B"
bash tools/gpu_ab_env.sh "$TAG/k2" bf16 2 down1_fwd,down2_fwd,up1_fwd,d2_fwd "- $B"
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- $B - $B"
echo "[r03u] done"
