#!/bin/bash
# Quick round-5 check: selected -m gpu tests and the default bench line (compact, full tables to a file).
#   bash tools/gpu_quick5.sh TAG "TEST SELECTION"
set -eo pipefail
TAG=${1:-q5}
SEL=${2:-tests/test_torch_ops_gpu.py tests/test_graph_gpu.py}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest $SEL -m gpu -x -q -rf --tb=short --timeout 120 --timeout-method thread \
    > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
step bench 400 python3 bench.py --full-out "gpurun_out/$TAG/bench_full.json" > "$O/bench.json" 2> "$O/bench.err"
wc -c "$O/bench.json"
cut -c1-600 "$O/bench.json"
