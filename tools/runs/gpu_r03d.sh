#!/bin/bash
# op16 (ABI 11) check-in: kernel parity of the operand-plane entries, the reduced-precision step
# tests, bench A/B (planes on / MRAGAN_NO_OP16=1), then the brick tile sweep in bf16.
set -eo pipefail
TAG=${1:-r03d}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 400 python -u -m pytest tests/test_kernels_gpu.py -v -rf --tb=short --timeout 120 --timeout-method thread \
    -k "op16 or brick_in_stats or wgrad3 or presplit or dgrad" > "$O/kt.log" 2>&1
tail -2 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
step st 600 python -u -m pytest tests/test_step_gpu.py -v -rf --tb=short --timeout 200 --timeout-method thread \
    -k "(bf16 or fp16) and not bf16x3" > "$O/st.log" 2>&1
tail -2 "$O/st.log"; grep -E "^FAILED" "$O/st.log" | head || true
bash tools/gpu_variants.sh "$TAG/var" "" "--single-stream"
MRAGAN_NO_OP16=1 bash tools/gpu_variants.sh "$TAG/var_noop16" ""
bash tools/gpu_brick_sweep.sh "$TAG/sweep" bf16 "-/0 128,128/0 128,128/1 128,128/2 128,64/0 64,128/0"
echo "[r03d] done"
