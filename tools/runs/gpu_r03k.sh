#!/bin/bash
set -eo pipefail
TAG=${1:-r03k}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 300 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "in_stats or conv3d or x3 or transpose" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
step st 600 python -u -m pytest tests/test_step_gpu.py -q -rf --tb=short --timeout 200 --timeout-method thread \
    -k "s64 or s128 or s32" > "$O/st.log" 2>&1
tail -1 "$O/st.log"; grep -E "^FAILED" "$O/st.log" | head || true
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- MRAGAN_NO_IN_STATS=1 MRAGAN_W3_BLOCKS=128 MRAGAN_W3_BLOCKS=192 MRAGAN_BRICK_CFG=128,128 -"
echo "[r03k] done"
