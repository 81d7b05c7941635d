#!/bin/bash
# r06v: stride-2 brick default variant 4 + thin weight gradients on 512 threads — kernel tests, graph bit
# identity, step suites (64³ b2, 96³, 128³, UNet), same-box step A/Bs (headline: MRAGAN_NO_BRICK_S2=1;
# UNet leg: MRAGAN_THIN_WGRAD_T=256)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06v
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "stride2 or thin or wgrad" > "$O/kern.log" 2>&1 || { tail -40 "$O/kern.log"; exit 1; }
tail -2 "$O/kern.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py > "$O/graph.log" 2>&1 || { tail -40 "$O/graph.log"; exit 1; }
tail -2 "$O/graph.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_step_gpu.py -k "s64_b2 or s128 or s96 or unet" > "$O/steps.log" 2>&1 || { tail -40 "$O/steps.log"; exit 1; }
tail -2 "$O/steps.log"
bash tools/gpu_envab.sh r06v/ab 3 "-" "MRAGAN_NO_BRICK_S2=1"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r06v/ab_unet 3 "-" "MRAGAN_THIN_WGRAD_T=256"
BENCH_ARGS="--size 128 --batch 1" bash tools/gpu_envab.sh r06v/ab_128 2 "-" "MRAGAN_NO_BRICK_S2=1"
