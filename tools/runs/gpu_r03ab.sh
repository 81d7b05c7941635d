#!/bin/bash
# r03ab: G head data gradient with the last up-conv IN's backward statistics (ABI 12);
# MRAGAN_NO_HEAD_STATS=1 = statistics pass.  Parity + step A/B.
set -eo pipefail
TAG=${1:-r03ab}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_graph_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "head_dgrad or in_stats or thin or step or graph" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head || true
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- MRAGAN_NO_HEAD_STATS=1 - MRAGAN_NO_HEAD_STATS=1"
echo "[r03ab] done"
