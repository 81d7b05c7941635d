#!/bin/bash
# split data gradient: kernel tests, then the 128³ b1 step with the split (default) and without
# (MRAGAN_DGRAD_SPLIT=0), alternating, same box
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bc}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "interior_shell or brick_conv_and_wgrad or in_launch_finalize or dgrad_backward_statistics" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
B="python3 bench.py --size 128 --batch 1 --legs= --no-cpu-baseline --alt-precisions= --no-kernel-timing --steps 10 --warmup 3"
for i in 1 2; do
  for side in split whole; do
    if [ $side = whole ]; then export MRAGAN_DGRAD_SPLIT=0; else unset MRAGAN_DGRAD_SPLIT; fi
    step "b128 $side $i" 300 $B --full-out "$O/full_${side}_$i.json" > "$O/b128_${side}_$i.json" 2> "$O/b128_${side}_$i.err"
    python3 -c "import json; d=json.loads(open('$O/b128_${side}_$i.json').read().strip().splitlines()[-1]); print('128 $side $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
