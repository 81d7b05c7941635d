#!/bin/bash
# GPU-box pass: selected parity tests only (short tracebacks), log under gpurun_out/TAG/.
#   bash tools/gpu_tests.sh TAG "pytest -k expr"
set -euo pipefail
TAG=${1:-t}
KEXPR=${2:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --tb=short --timeout 300 --timeout-method thread -k "$KEXPR" 2>&1 | tee "$O/pytest.log"
