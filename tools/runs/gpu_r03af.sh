#!/bin/bash
# r03af: backward-statistics tests + the default bench line at HEAD
set -eo pipefail
TAG=${1:-r03af}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_step_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "backward_statistics or in_stats or x3 or step" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head || true
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
step bench 700 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "[r03af] done"
