#!/bin/bash
# Kernel trace of the bench step:  bash tools/gpu_trace.sh TAG PRECISION [extra bench args]
set -eo pipefail
TAG=$1; PREC=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --precision "$PREC" --steps 10 --warmup 3 --no-cpu-baseline "$@" > "$O/trace.log" 2>&1
grep '^{' "$O/trace.log" | head -1 | cut -c1-300
