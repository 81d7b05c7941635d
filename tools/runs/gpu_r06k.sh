#!/bin/bash
# r06k: rocprofv3 kernel trace of the replayed headline step at HEAD (4 streams: lanes 0/1, the
# D side streams) for the lane / idle analysis
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06k
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-kernel-timing --alt-precisions '' --legs '' --no-cpu-baseline \
    --full-out '' > "$O/trace.log" 2>&1
grep '^{' "$O/trace.log" | cut -c1-200
