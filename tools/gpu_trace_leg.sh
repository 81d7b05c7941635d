#!/bin/bash
# Kernel trace (graph replay) of one bench workload:  bash tools/gpu_trace_leg.sh TAG [bench args...]
set -eo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-kernel-timing --alt-precisions '' --legs '' --no-cpu-baseline \
    --full-out '' "$@" > "$O/trace.log" 2>&1
grep '^{' "$O/trace.log" | cut -c1-300
CSV=$(find "$O/trace" -name '*kernel_trace.csv' | head -1)
python3 "$R/tools/prof_summary.py" "$CSV" --steps 13 --top 60 > "$O/summary.md" 2>&1 || true
head -30 "$O/summary.md"
