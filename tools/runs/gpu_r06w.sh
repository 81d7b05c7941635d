#!/bin/bash
# r06w: stride-2 brick on G down2 only (down1 back on the implicit GEMM) — kernel tests (default and forced
# variants in child processes), graph bit identity, same-box A/Bs at 64³ b2 and 128³ b1; UNet wgrad_small
# threshold 32 vs 64
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06w
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "stride2" > "$O/kern.log" 2>&1 || { tail -40 "$O/kern.log"; exit 1; }
tail -2 "$O/kern.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py -k "stride2 or headline" > "$O/graph.log" 2>&1 || { tail -40 "$O/graph.log"; exit 1; }
tail -2 "$O/graph.log"
bash tools/gpu_envab.sh r06w/ab 2 "-" "MRAGAN_NO_BRICK_S2=1"
BENCH_ARGS="--size 128 --batch 1" bash tools/gpu_envab.sh r06w/ab_128 2 "-" "MRAGAN_NO_BRICK_S2=1"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r06w/ab_unet 2 "-" "MRAGAN_WGRAD_SMALL_M=32"
