#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02h
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 900 python -u -m pytest tests -m gpu -q --tb=short --timeout 300 --timeout-method thread -k "instnorm or graph_step or (step_gpu and (s32 or s24)) or sliding or checkpoint" > "$O/pytest.log" 2>&1
tail -15 "$O/pytest.log"
step bench 400 python3 bench.py --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
