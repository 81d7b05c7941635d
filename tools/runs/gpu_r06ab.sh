#!/bin/bash
# r06ab: generator weight repack at the end of each lane (after its Adam) instead of at the next step's
# start — graph / step / checkpoint / DP suites, smoke, same-box A/B (MRAGAN_PACK_AT_START=1)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06ab
mkdir -p "$O"
cd "$R"
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py tests/test_checkpoint_gpu.py tests/test_dp_gpu.py > "$O/graph.log" 2>&1 || { tail -40 "$O/graph.log"; exit 1; }
tail -2 "$O/graph.log"
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_step_gpu.py > "$O/steps.log" 2>&1 || { tail -40 "$O/steps.log"; exit 1; }
tail -2 "$O/steps.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
bash tools/gpu_envab.sh r06ab/ab 3 "-" "MRAGAN_PACK_AT_START=1"
BENCH_ARGS="--size 128 --batch 1" bash tools/gpu_envab.sh r06ab/ab_128 2 "-" "MRAGAN_PACK_AT_START=1"
