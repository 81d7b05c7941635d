#!/bin/bash
# Round-5 check: kernel tests (-k KEXPR), step tests (-k SEXPR), then the default bench line.
#   bash tools/gpu_check5.sh TAG "KEXPR" "SEXPR" [nobench]
set -eo pipefail
TAG=$1; KEXPR=$2; SEXPR=$3; NOBENCH=${4:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
if [ -n "$KEXPR" ]; then
  step ktests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf --tb=short --timeout 120 \
      --timeout-method thread -k "$KEXPR" > "$O/ktests.log" 2>&1
  tail -3 "$O/ktests.log"
fi
if [ -n "$SEXPR" ]; then
  step stests 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short --timeout 300 \
      --timeout-method thread -k "$SEXPR" > "$O/stests.log" 2>&1
  tail -3 "$O/stests.log"
fi
if [ -z "$NOBENCH" ]; then
  step bench 500 python3 bench.py --full-out "gpurun_out/$TAG/bench_full.json" > "$O/bench.json" 2> "$O/bench.err"
  wc -c "$O/bench.json"
  cut -c1-300 "$O/bench.json"
fi
