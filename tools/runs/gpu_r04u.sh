#!/bin/bash
# r04u: the TG 64 fix of wgrad3s2's 16-bit gathered operand (the 33rd fine position) — kernel
# tests, the plane-vs-fp32 step A/B at 64^3 (both layers), the reduced-precision step subset,
# then the PMC passes of r04t
set -eo pipefail
TAG=${1:-r04u}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "stride2 or op16 or wgrad_s2" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step planes 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py \
  -k "stride2_planes" > "$O/planes.log" 2>&1
tail -2 "$O/planes.log"
step stepp 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "bf16 or fp16" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
bash tools/gpu_r04t.sh r04u_pmc
echo "[r04u] done"
