#!/bin/bash
# r05ac: wide brickT only on large grids (UNet regression), one-split wgrad back on slab + reduce —
# tests, UNet / headline A/B, UNet trace
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05ac
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "brickT or stride2 or bf16x3_wgrad or transpose" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
BENCH_ARGS="--size 64 --batch 1 --netG unet_custom" bash tools/gpu_envab.sh r05ac/unet 2 "-" "MRAGAN_BRICKT_WIDE=0" "MRAGAN_BRICKT_WIDE=1"
bash tools/gpu_envab.sh r05ac/head 2 "-" "MRAGAN_BRICKT_WIDE=0"
bash tools/gpu_trace_leg.sh r05ac/unet_trace --size 64 --batch 1 --netG unet_custom
