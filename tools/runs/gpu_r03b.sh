#!/bin/bash
# reduced-precision step tests vs the rounded-operand oracle + a bf16 bench breakdown
set -eo pipefail
TAG=${1:-r03b}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step steptests 600 python -u -m pytest tests/test_step_gpu.py -m gpu -v -s -rf --tb=short --timeout 300 \
    --timeout-method thread -k "(bf16 and not bf16x3) or fp16" > "$O/pytest.log" 2>&1
tail -4 "$O/pytest.log"
step bench 400 python3 bench.py --precision bf16 --alt-precisions '' --legs '' --no-cpu-baseline > "$O/bench_bf16.json" 2> "$O/bench_bf16.err"
cut -c1-300 "$O/bench_bf16.json"
