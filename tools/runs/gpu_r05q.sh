#!/bin/bash
# r05q: small-instance InstanceNorm restricted to full-line channel slices — IN tests, per-shape
# timing on / off, same-box step A/B (UNet leg, headline)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05q
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "instnorm or in_stats or in_launch" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
step inb0 120 env MRAGAN_IN_SMALL=0 python3 tools/in_bench.py > "$O/inb0.txt" 2>&1
step inb1 120 python3 tools/in_bench.py > "$O/inb1.txt" 2>&1
paste "$O/inb0.txt" "$O/inb1.txt" | cut -c1-200
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r05q/unet 2 "-" "MRAGAN_IN_SMALL=0"
bash tools/gpu_envab.sh r05q/head 2 "-" "MRAGAN_IN_SMALL=0"
