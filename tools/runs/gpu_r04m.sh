#!/bin/bash
# r04m: res-block data gradient variants (K-split brick forced vs the 8-wave brick) at the three
# legs' shapes, with and without the backward-statistics epilogue; forward for reference
set -eo pipefail
TAG=${1:-r04m}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
KB="python3 tools/kbench.py --ops res_fwd16,res_dgrad16,res_dgrad16s,res_wgrad16 --reps 30 --precision bf16"
for shp in "--S 64 --N 4" "--S 64 --N 2" "--S 128 --N 2" "--S 96 --N 2"; do
  for v in 0 1 2 3; do
    if [ $v = 0 ]; then unset MRAGAN_BRICK_KS; else export MRAGAN_BRICK_KS=$v; fi
    echo "== $shp KS=$v"
    step kb 120 $KB $shp
  done
done
unset MRAGAN_BRICK_KS
echo "[r04m] done"
