#!/bin/bash
set -eo pipefail
TAG=${1:-r03l}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 300 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "in_stats or wgrad" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- MRAGAN_W3_BLOCKS=160 MRAGAN_W3_BLOCKS=224 MRAGAN_BRICK_CFG=128,128 MRAGAN_IG_MINBLOCKS=256 MRAGAN_IG_MINBLOCKS=1024 MRAGAN_W3S2_BUDGET=50 MRAGAN_W3S2_BUDGET=75 -"
echo "[r03l] done"
