#!/bin/bash
# r06i: in-launch IN finalize in the 8-wave brick (the 18³ data gradient at N = 4) and the
# discriminator repacks on the side streams: kernel / graph / step tests, same-box A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06i
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kern 400 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf --tb=short --timeout 120 --timeout-method thread \
    > "$O/kern.log" 2>&1
tail -3 "$O/kern.log"
step graph 600 python3 -u -m pytest tests/test_graph_gpu.py tests/test_dp_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 \
    --timeout-method thread > "$O/graph.log" 2>&1
tail -3 "$O/graph.log"
step steps 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread \
    > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
bash tools/gpu_envab.sh r06i/ab 3 "-" "MRAGAN_NO_X3_FIN=1"
