#!/bin/bash
# r06p: D_A's work (frozen pass, D phase, Adam) forked onto side 0 right after G_A's first pass,
# beside the cycle-pass forwards — graph / step suites, then same-box A/B against MRAGAN_LATE_D=1
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06p
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py tests/test_step_gpu.py tests/test_dp_gpu.py > "$O/steps.log" 2>&1
tail -2 "$O/steps.log"
bash tools/gpu_envab.sh r06p/ab 3 "-" "MRAGAN_LATE_D=1"
