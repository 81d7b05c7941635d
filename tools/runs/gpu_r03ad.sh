#!/bin/bash
# r03ad: stride-2 data gradients with the next IN's backward statistics (ABI 12);
# MRAGAN_NO_S2_STATS=1 = statistics pass.  Parity + step A/B.
set -eo pipefail
TAG=${1:-r03ad}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py tests/test_graph_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "backward_statistics" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head || true
true
echo "[r03ad] done"
