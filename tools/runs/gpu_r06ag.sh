#!/bin/bash
# r06ag: 1024-thread k4 thin weight gradients (A/B form) — thin kernel tests in both forms, UNet-leg A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06ag
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "thin" > "$O/kern.log" 2>&1 || { tail -30 "$O/kern.log"; exit 1; }
tail -1 "$O/kern.log"
MRAGAN_THIN_WGRAD_T=1024 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "thin" > "$O/kern1024.log" 2>&1 || { tail -30 "$O/kern1024.log"; exit 1; }
tail -1 "$O/kern1024.log"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r06ag/ab_unet 3 "-" "MRAGAN_THIN_WGRAD_T=1024"
