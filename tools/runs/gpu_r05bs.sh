#!/bin/bash
# fp32-pack refresh unit test + the 128³ / 96³ step gates after the fp32-input block-path refresh
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bs}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "fresh_fp32 or interior_shell or s128 or s96" > "$O/tests.log" 2>&1
tail -3 "$O/tests.log"
