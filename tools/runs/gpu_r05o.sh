#!/bin/bash
# r05o: single-launch InstanceNorm for small instances — IN kernel tests, step parity subset,
# same-box A/B (UNet leg, headline)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05o
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "instnorm or in_stats or in_launch" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
step steptests 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -x -q -rf --tb=short --timeout 300 \
    --timeout-method thread -k "unet_s32 or s32_b2 or unet_s64" > "$O/step.log" 2>&1
tail -3 "$O/step.log"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r05o/unet 2 "-" "MRAGAN_IN_SMALL=0"
bash tools/gpu_envab.sh r05o/head 2 "-" "MRAGAN_IN_SMALL=0"
