#!/bin/bash
# r06s: short-contraction weight gradient (wgrad_small_kernel) — kernel tests, UNet step suites, same-box
# UNet-leg A/B of the contraction threshold (0 = off, 64 = default, 128)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06s
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "wgrad" > "$O/kern.log" 2>&1 || { tail -30 "$O/kern.log"; exit 1; }
tail -2 "$O/kern.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_step_gpu.py -k "unet" > "$O/steps.log" 2>&1 || { tail -30 "$O/steps.log"; exit 1; }
tail -2 "$O/steps.log"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r06s/ab_unet 3 "-" "MRAGAN_WGRAD_SMALL_M=0" "MRAGAN_WGRAD_SMALL_M=128"
