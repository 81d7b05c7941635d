#!/bin/bash
set -eo pipefail
TAG=${1:-r03o}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 300 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "instnorm" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
bash tools/gpu_ab_env.sh "$TAG/in" bf16 4 in_bwd,in_bwd16 "- MRAGAN_IN_CONTIG_ROWS=1"
bash tools/gpu_stepenv_ab.sh "$TAG/ab" "- MRAGAN_IN_CONTIG_ROWS=1 -"
echo "[r03o] done"
