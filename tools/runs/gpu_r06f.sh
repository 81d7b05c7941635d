#!/bin/bash
# r06f: frozen discriminator passes on the side streams (beside the cycle-pass backwards): graph
# tests, the step suites, same-box A/B against the frozen passes on the lanes and the two-phase step
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06f
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step graph 600 python3 -u -m pytest tests/test_graph_gpu.py tests/test_dp_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 \
    --timeout-method thread > "$O/graph.log" 2>&1
tail -3 "$O/graph.log"
step steps 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread \
    > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
bash tools/gpu_envab.sh r06f/ab 3 "-" "MRAGAN_FROZEN_D_ON_LANES=1"
