#!/bin/bash
set -eo pipefail
TAG=${1:-r03n}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 300 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "instnorm or in_stats or op16 or pack" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
step st 600 python -u -m pytest tests/test_step_gpu.py tests/test_graph_gpu.py -q -rf --tb=short --timeout 200 --timeout-method thread \
    > "$O/st.log" 2>&1
tail -1 "$O/st.log"; grep -E "^FAILED" "$O/st.log" | head || true
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- MRAGAN_IN_FINALIZE_LAUNCH=1 MRAGAN_FP32_PACKS=1 - MRAGAN_IN_FINALIZE_LAUNCH=1;MRAGAN_FP32_PACKS=1"
echo "[r03n] done"
