#!/bin/bash
# 96³ b1 nc2 fp16 step (BASELINE configs[4]'s per-GPU unit) with the skip-gradient statistics
# (default) and without (MRAGAN_NO_SKIP_STATS=1), alternating, same box
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bl}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
B="python3 bench.py --size 96 --batch 1 --nc 2 --precision fp16 --legs= --no-cpu-baseline --alt-precisions= --no-kernel-timing --steps 10 --warmup 3"
for i in 1 2; do
  for side in skip noskip; do
    if [ $side = noskip ]; then export MRAGAN_NO_SKIP_STATS=1; else unset MRAGAN_NO_SKIP_STATS; fi
    step "b96 $side $i" 300 $B --full-out "$O/full_${side}_$i.json" > "$O/b96_${side}_$i.json" 2> "$O/b96_${side}_$i.err"
    python3 -c "import json; d=json.loads(open('$O/b96_${side}_$i.json').read().strip().splitlines()[-1]); print('96 $side $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
