#!/bin/bash
# r06d: the 64³ b2 step suite with the regenerated 2-step precision fixture (step 1 = the first
# graph replay, gated against the oracle in bf16 / fp16 / bf16x3); a rocprofv3 kernel trace of the
# replayed headline step (real in-step kernel durations, two lanes)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06d
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step steps 600 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 --timeout-method thread \
    -k "s64_b2" > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
cd /tmp && export TMPDIR=/tmp
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-kernel-timing --alt-precisions '' --legs '' --no-cpu-baseline \
    --full-out '' > "$O/trace.log" 2>&1
grep '^{' "$O/trace.log" | cut -c1-200
