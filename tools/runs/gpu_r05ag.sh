#!/bin/bash
# r05ag: InstanceNorm loads issued ahead of the waits (paired voxels, branch-free selects) — tests,
# headline / UNet / 128³ A/B against the previous instnorm.hip (variant build inbase)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05ag
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "instnorm or in_small or IN or rpad or stride2 or op16" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
step steptests 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -x -q -rf --tb=short --timeout 300 \
    --timeout-method thread -k "s64_b2 or s32_b1 or unet" > "$O/step.log" 2>&1
tail -3 "$O/step.log"
grep -q " failed" "$O/step.log" && exit 1
B="MRAGAN_HIP_LIB=$R/mra-gan_amd/lib/var/inbase/libmragan_hip.so"
bash tools/gpu_envab.sh r05ag/head 3 "-" "$B"
BENCH_ARGS="--size 64 --batch 1 --netG unet_custom" bash tools/gpu_envab.sh r05ag/unet 2 "-" "$B"
BENCH_ARGS="--size 128 --batch 1" bash tools/gpu_envab.sh r05ag/l128 2 "-" "$B"
