#!/bin/bash
set -eo pipefail
TAG=${1:-r03g}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 400 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread \
    > "$O/kt.log" 2>&1
tail -2 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
bash tools/gpu_ab_env.sh "$TAG/w4" bf16 4 res_wgrad16,res_wgrad "- MRAGAN_W3_NO_AL=1"
bash tools/gpu_ab_env.sh "$TAG/ig" bf16 4 down1_fwd,down2_fwd,up1_fwd,d2_fwd "-"
step st 700 python -u -m pytest tests/test_step_gpu.py -q -rf --tb=short --timeout 200 --timeout-method thread \
    > "$O/st.log" 2>&1
tail -2 "$O/st.log"; grep -E "^FAILED" "$O/st.log" | head || true
bash tools/gpu_variants.sh "$TAG/var" "" "--precision bf16x3"
echo "[r03g] done"
