#!/bin/bash
# r06e: the D phase beside the G backward (single GPU, one graph): graph-vs-eager and
# overlapped-vs-two-phase bit identity, the step suites, the DP tests, same-box step A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06e
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step graph 600 python3 -u -m pytest tests/test_graph_gpu.py tests/test_dp_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 \
    --timeout-method thread > "$O/graph.log" 2>&1
tail -3 "$O/graph.log"
step steps 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread \
    > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
bash tools/gpu_envab.sh r06e/ab 2 "-" "MRAGAN_TWO_PHASE=1"
