#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02m
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 1000 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread -k "sampler or s96 or instnorm or thin" > "$O/pytest.log" 2>&1
tail -12 "$O/pytest.log"
