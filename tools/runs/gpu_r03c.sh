#!/bin/bash
# kernel tests + reduced-precision step tests + bf16 / bf16x3 bench breakdowns
set -eo pipefail
TAG=${1:-r03c}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kernels 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf --tb=short --timeout 200 \
    --timeout-method thread > "$O/kernels.log" 2>&1
tail -3 "$O/kernels.log"
grep -E "FAILED|ERROR" "$O/kernels.log" | head -20 || true
step steptests 600 python -u -m pytest tests/test_step_gpu.py -m gpu -v -s -rf --tb=short --timeout 300 \
    --timeout-method thread -k "(bf16 and not bf16x3) or fp16" > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
step bench16 300 python3 bench.py --precision bf16 --alt-precisions bf16x3 --legs '' --no-cpu-baseline > "$O/bench_bf16.json" 2> "$O/bench_bf16.err"
cut -c1-300 "$O/bench_bf16.json"
