#!/bin/bash
# Full GPU test suite (the driver's round-end tier), log under gpurun_out/TAG/.
set -eo pipefail
TAG=${1:-full}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 1100 python -u -m pytest tests -m gpu -v -rf --tb=short --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -15 "$O/pytest.log"
