#!/bin/bash
# r05af: small InstanceNorm kernels with 4 voxels' loads in flight — tests, UNet / headline A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05af
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "instnorm or in_small or IN" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
BENCH_ARGS="--size 64 --batch 1 --netG unet_custom" bash tools/gpu_envab.sh r05af/unet 2 "-" "MRAGAN_IN_SMALL=0"
bash tools/gpu_trace_leg.sh r05af/unet_trace --size 64 --batch 1 --netG unet_custom
