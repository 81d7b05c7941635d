#!/bin/bash
# r05ah: in-tree = small-IN batching only; variants inbase (previous instnorm.hip) and inpairs
# (paired voxels, conditional optional loads) — IN tests, headline / UNet A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05ah
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "instnorm" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
B="MRAGAN_HIP_LIB=$R/mra-gan_amd/lib/var/inbase/libmragan_hip.so"
P="MRAGAN_HIP_LIB=$R/mra-gan_amd/lib/var/inpairs/libmragan_hip.so"
bash tools/gpu_envab.sh r05ah/head 3 "-" "$B" "$P"
BENCH_ARGS="--size 64 --batch 1 --netG unet_custom" bash tools/gpu_envab.sh r05ah/unet 2 "-" "$B" "$P"
