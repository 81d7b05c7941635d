#!/bin/bash
# 128³ b1 step: conv2 data gradient with IN1 statistics (default) vs split dgrad + statistics pass (MRAGAN_IN1_SPLIT=1),
# alternating, same box; then the kbench res data gradients at 128³ N = 2
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bg}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
B="python3 bench.py --size 128 --batch 1 --legs= --no-cpu-baseline --alt-precisions= --no-kernel-timing --steps 10 --warmup 3"
for i in 1 2; do
  for side in stats split; do
    if [ $side = split ]; then export MRAGAN_IN1_SPLIT=1; else unset MRAGAN_IN1_SPLIT; fi
    step "b128 $side $i" 300 $B --full-out "$O/full_${side}_$i.json" > "$O/b128_${side}_$i.json" 2> "$O/b128_${side}_$i.err"
    python3 -c "import json; d=json.loads(open('$O/b128_${side}_$i.json').read().strip().splitlines()[-1]); print('128 $side $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
