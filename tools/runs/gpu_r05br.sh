#!/bin/bash
# split data gradient with its fp32 pack refreshed: the step suite (all sizes), then the 128³ step
# default (split) vs MRAGAN_DGRAD_SPLIT=0, alternating
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bq}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step steptests 600 python -u -m pytest tests/test_step_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/steptests.log" 2>&1
tail -3 "$O/steptests.log"
grep -q "failed" "$O/steptests.log" && exit 1
B="python3 bench.py --size 96 --batch 1 --nc 2 --precision fp16 --legs= --no-cpu-baseline --alt-precisions= --no-kernel-timing --steps 10 --warmup 3"
for i in 1 2; do
  for side in split whole; do
    if [ $side = whole ]; then export MRAGAN_DGRAD_SPLIT=0; else unset MRAGAN_DGRAD_SPLIT; fi
    step "b96 $side $i" 300 $B --full-out "$O/full_${side}_$i.json" > "$O/b96_${side}_$i.json" 2> "$O/b96_${side}_$i.err"
    python3 -c "import json; d=json.loads(open('$O/b96_${side}_$i.json').read().strip().splitlines()[-1]); print('96 $side $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
