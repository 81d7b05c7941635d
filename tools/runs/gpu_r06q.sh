#!/bin/bash
# r06q: stream priorities — lanes (capture stream, lane 1) high, D side streams low (MRAGAN_LANE_PRIO=1)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
MRAGAN_LANE_PRIO=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py -k "overlapped or eager" > gpurun_out/r06q_graph.log 2>&1 || { tail -20 gpurun_out/r06q_graph.log; exit 1; }
tail -1 gpurun_out/r06q_graph.log
bash tools/gpu_envab.sh r06q/ab 3 "-" "MRAGAN_LANE_PRIO=1"
