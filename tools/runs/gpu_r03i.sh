#!/bin/bash
# Same-box step A/B of this round's kernel work (all A/B switches off vs on), then a clean kernel
# trace of the headline workload.
set -eo pipefail
TAG=${1:-r03i}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 300 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "x3 or conv or op16" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"
bash tools/gpu_variants.sh "$TAG/on" "" ""
MRAGAN_NO_OP16=1 MRAGAN_NO_IN_STATS=1 MRAGAN_W3_NO_AL=1 MRAGAN_NO_TILE8=1 bash tools/gpu_variants.sh "$TAG/off" "" ""
bash tools/gpu_variants.sh "$TAG/on2" ""
cd /tmp && export TMPDIR=/tmp
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-kernel-timing --alt-precisions '' --legs '' --no-cpu-baseline \
    > "$O/trace.log" 2>&1
echo "[r03i] done"
