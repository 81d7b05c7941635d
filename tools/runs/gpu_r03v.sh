#!/bin/bash
# r03v: tests at HEAD-in-progress + PMC probe (stalls, MFMA, traffic) of the stride-2 kernels
set -eo pipefail
TAG=${1:-r03v}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "x3 or igemm or in_stats or conv" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head || true
PREC=bf16 KN=4 bash tools/pmc_probe.sh "$TAG/pmc" down1_wgrad,up2_fwd,down1_fwd,down2_wgrad
echo "[r03v] done"
