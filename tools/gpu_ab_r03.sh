#!/bin/bash
# A/B of kernel variants at the bench shapes (bf16): brick tiles, the dgrad interior/shell split
set -eo pipefail
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
KB="python3 tools/kbench.py --ops res_fwd,res_dgrad,res_wgrad,in_bwd,in_bwd16,in_fwd16 --reps 40 --precision bf16"
for N in 4 2; do
  step base$N 120 $KB --N $N > "$O/base_N$N.log" 2>&1
  for cfg in 128,128 128,64 64,128 64,64; do
    step cfg$cfg$N 120 env MRAGAN_BRICK_CFG=$cfg $KB --N $N > "$O/cfg_${cfg}_N$N.log" 2>&1
  done
  step split$N 120 env MRAGAN_DGRAD_SPLIT=1 $KB --N $N > "$O/split_N$N.log" 2>&1
done
for f in "$O"/*.log; do echo "== $(basename $f)"; grep "us/call" "$f" || true; done
