#!/bin/bash
# r06h: Adam updates inside the overlapped step (each network's at the end of the stream that
# finished its gradients): graph / DP / step suites (incl. the 128³ bf16x3 fixture's new fp32
# realisations), same-box A/B against the four Adams after the graph
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06h
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step graph 600 python3 -u -m pytest tests/test_graph_gpu.py tests/test_dp_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 \
    --timeout-method thread > "$O/graph.log" 2>&1
tail -3 "$O/graph.log"
step steps 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 --timeout-method thread \
    > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
bash tools/gpu_envab.sh r06h/ab 3 "-" "MRAGAN_ADAM_AFTER=1"
