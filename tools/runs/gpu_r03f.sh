#!/bin/bash
set -eo pipefail
TAG=${1:-r03f}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 300 python -u -m pytest tests/test_kernels_gpu.py -v -rf --tb=short --timeout 120 --timeout-method thread \
    -k "wgrad or op16 or bf16x3_fwd_dgrad or brick" > "$O/kt.log" 2>&1
tail -2 "$O/kt.log"; grep -E "^FAILED" "$O/kt.log" | head || true
bash tools/gpu_ab_env.sh "$TAG/ab4" bf16 4 res_wgrad16,res_wgrad "- MRAGAN_W3_NO_AL=1"
bash tools/gpu_ab_env.sh "$TAG/ab2" bf16 2 res_wgrad16 "- MRAGAN_W3_NO_AL=1"
bash tools/gpu_ab_env.sh "$TAG/brick4" bf16 4 res_fwd16,res_dgrad16,res_fwd,res_dgrad "-"
bash tools/gpu_ab_env.sh "$TAG/brick2" bf16 2 res_fwd16,res_dgrad16 "-"
bash tools/gpu_variants.sh "$TAG/var" ""
echo "[r03f] done"
