#!/bin/bash
# op16 backward-statistics + D-first tile check-in, then PMC of the op16 res-block kernels (bf16).
set -eo pipefail
TAG=${1:-r03e}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 400 python -u -m pytest tests/test_kernels_gpu.py -v -rf --tb=short --timeout 120 --timeout-method thread \
    -k "op16 or dgrad or thin" > "$O/kt.log" 2>&1
tail -2 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
step st 600 python -u -m pytest tests/test_step_gpu.py -v -rf --tb=short --timeout 200 --timeout-method thread \
    -k "(bf16 or fp16) and not bf16x3" > "$O/st.log" 2>&1
tail -2 "$O/st.log"; grep -E "^FAILED" "$O/st.log" | head || true
bash tools/gpu_variants.sh "$TAG/var" ""
PREC=bf16 step pmc 400 bash tools/pmc_probe.sh "$TAG/pmc" res_fwd16,res_dgrad16,res_wgrad16
echo "[r03e] done"
