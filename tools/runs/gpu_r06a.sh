#!/bin/bash
# r06a: ABI 19 (shell pass on the pre-split weights, no stale fp32 pack handed to the library):
# the split / pack kernel tests, the graph-vs-eager tests incl. the headline dispatch, the step
# suites of the split sizes (96³ nc2, 128³), a quick headline bench
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06a
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kern 300 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "interior_shell or null_fp32 or stale_fp32 or skip_statistics or op16_res or presplit" > "$O/kern.log" 2>&1
tail -3 "$O/kern.log"
step graph 600 python3 -u -m pytest tests/test_graph_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 --timeout-method thread \
    > "$O/graph.log" 2>&1
tail -3 "$O/graph.log"
step steps 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread \
    -k "s96 or s128" > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
step bench 300 python3 bench.py --steps 30 --warmup 5 --alt-precisions '' --no-cpu-baseline --full-out "gpurun_out/r06a/bench_full.json" \
    > "$O/bench.json" 2> "$O/bench.err"
cut -c1-300 "$O/bench.json"
