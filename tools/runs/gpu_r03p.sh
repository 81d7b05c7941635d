#!/bin/bash
# r03p: uniform buffer descriptors (no waterfall loops in conv_brick_x3) and the one-plane brick
# prefetch distances, as variant libraries on one box: kernel A/B + step A/B.
set -eo pipefail
TAG=${1:-r03p}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 400 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "brick or op16 or thinn or thin1 or wgrad" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
L=mra-gan_amd/lib/ab
SETS="MRAGAN_HIP_LIB=$L/base/libmragan_hip.so - MRAGAN_HIP_LIB=$L/kpf18/libmragan_hip.so MRAGAN_HIP_LIB=$L/kad5/libmragan_hip.so"
bash tools/gpu_ab_env.sh "$TAG/k" bf16 4 res_fwd16,res_dgrad16,res_fwd,res_dgrad "$SETS"
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "$SETS MRAGAN_HIP_LIB=$L/base/libmragan_hip.so -"
echo "[r03p] done"
