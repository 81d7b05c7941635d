#!/bin/bash
# r06o: implicit-GEMM split-K reduced in the launch (tickets; as run: fused by default, MRAGAN_NO_SK_FUSE=1
# the reduce launch — after this run the fusion is opt-in, MRAGAN_SK_FUSE=1) — kernel tests (bit identity against
# the reduce launch in a child process), step suites, then same-box A/B on the UNet leg and the headline
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06o
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "splitk or bf16x3_fwd_dgrad or conv3d_fwd or stride2 or igemm" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py tests/test_step_gpu.py > "$O/steps.log" 2>&1
tail -2 "$O/steps.log"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r06o/ab_unet 3 "-" "MRAGAN_NO_SK_FUSE=1"
bash tools/gpu_envab.sh r06o/ab 2 "-" "MRAGAN_NO_SK_FUSE=1"
