#!/bin/bash
# focused debugging: graph tests and the 64³ f32 step, with and without the capture cache
set -eo pipefail
TAG=${1:-dbg}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
export PYTHONFAULTHANDLER=1
step graph 300 python -u -m pytest tests/test_graph_gpu.py -m gpu -v -s -rf --tb=long --timeout 200 \
    --timeout-method thread > "$O/graph.log" 2>&1
tail -3 "$O/graph.log"
step s64f32_nocache 300 env MRAGAN_NO_GRAPH_CACHE=1 python -u -m pytest tests/test_step_gpu.py -m gpu -v -s -rf \
    --tb=long --timeout 200 --timeout-method thread -k "step_r9_s64_b2-f32" > "$O/s64_nocache.log" 2>&1
tail -3 "$O/s64_nocache.log"
step s64f32 300 python -u -m pytest tests/test_step_gpu.py -m gpu -v -s -rf --tb=long --timeout 200 \
    --timeout-method thread -k "step_r9_s64_b2-f32" > "$O/s64.log" 2>&1
tail -3 "$O/s64.log"
step f32all 600 python -u -m pytest tests/test_step_gpu.py -m gpu -v -rf --tb=long --timeout 200 \
    --timeout-method thread -k "f32" > "$O/f32all.log" 2>&1
tail -3 "$O/f32all.log"
echo "[dbg] done"
