#!/bin/bash
# r04g: step parity (every case × precision, bf16x3 against its emulation, tightened outlier
# budget) with the K-split brick; kernel tests; K-split phase stamps (kernel-argument placement)
set -eo pipefail
TAG=${1:-r04g}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step st 900 python -u -m pytest tests/test_step_gpu.py -q -s -rf --tb=short --timeout 600 --timeout-method thread > "$O/st.log" 2>&1
grep -E "passed|failed" "$O/st.log" | tail -1; grep -E "^FAILED" "$O/st.log" | head -30 || true
grep -E "over their envelope|vs emulation|loss rel err" "$O/st.log" > "$O/st_gates.txt" || true
step kt 600 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head -10 || true
MRAGAN_BRICK_KS=1 step "stamps" 200 python3 tools/diag_ks.py bf16 > "$O/stamps.txt" 2>&1
grep -v amdgpu.ids "$O/stamps.txt"
HIP_FORCE_DEV_KERNARG=1 MRAGAN_BRICK_KS=1 step "stamps devk" 200 python3 tools/diag_ks.py bf16 > "$O/stamps_devk.txt" 2>&1
grep -v amdgpu.ids "$O/stamps_devk.txt"
echo "[r04g] done"
