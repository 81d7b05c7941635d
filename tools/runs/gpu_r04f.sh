#!/bin/bash
# r04f: K-split brick phase stamps with / without device-memory kernel arguments
set -eo pipefail
TAG=${1:-r04f}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
MRAGAN_BRICK_KS=1 step "stamps" 200 python3 tools/diag_ks.py bf16 > "$O/stamps.txt" 2>&1
grep -v amdgpu.ids "$O/stamps.txt"
HIP_FORCE_DEV_KERNARG=1 MRAGAN_BRICK_KS=1 step "stamps devk" 200 python3 tools/diag_ks.py bf16 > "$O/stamps_devk.txt" 2>&1
grep -v amdgpu.ids "$O/stamps_devk.txt"
HIP_FORCE_DEV_KERNARG=0 MRAGAN_BRICK_KS=1 step "stamps hostk" 200 python3 tools/diag_ks.py bf16 > "$O/stamps_hostk.txt" 2>&1
grep -v amdgpu.ids "$O/stamps_hostk.txt"
echo "[r04f] done"
