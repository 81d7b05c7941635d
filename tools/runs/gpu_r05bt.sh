#!/bin/bash
# skip-gradient statistics at every batch (default) vs only N <= 2 (MRAGAN_SKIP_STATS_MAXN=2), 64³ b2 step alternating
# with them (default) and without (MRAGAN_SKIP_STATS_MAXN=2), alternating, same box
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05be}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step ktests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "skip_statistics" > "$O/ktests.log" 2>&1
tail -3 "$O/ktests.log"
grep -q " passed" "$O/ktests.log" && ! grep -q "failed" "$O/ktests.log" || { echo "kernel tests failed"; grep -E "FAILED|Error|assert" "$O/ktests.log" | head -20; exit 1; }
true
true
B="python3 bench.py --legs= --no-cpu-baseline --alt-precisions= --no-kernel-timing --steps 20 --warmup 5"
for i in 1 2 3; do
  for side in skip n2only; do
    if [ $side = n2only ]; then export MRAGAN_SKIP_STATS_MAXN=2; else unset MRAGAN_SKIP_STATS_MAXN; fi
    step "b64 $side $i" 300 $B --full-out "$O/full_${side}_$i.json" > "$O/b64_${side}_$i.json" 2> "$O/b64_${side}_$i.err"
    python3 -c "import json; d=json.loads(open('$O/b64_${side}_$i.json').read().strip().splitlines()[-1]); print('64 $side $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
