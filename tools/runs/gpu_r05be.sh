#!/bin/bash
# ABI 18 skip-gradient statistics: kernel tests, the step suite, then the 64³ b2 headline step
# with them (default) and without (MRAGAN_NO_SKIP_STATS=1), alternating, same box
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05be}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step ktests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "skip_statistics or stride2_dgrad_backward or dgrad_backward_statistics" > "$O/ktests.log" 2>&1
tail -3 "$O/ktests.log"
grep -q " passed" "$O/ktests.log" && ! grep -q "failed" "$O/ktests.log" || { echo "kernel tests failed"; grep -E "FAILED|Error|assert" "$O/ktests.log" | head -20; exit 1; }
step steptests 600 python -u -m pytest tests/test_step_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/steptests.log" 2>&1
tail -3 "$O/steptests.log"
B="python3 bench.py --legs= --no-cpu-baseline --alt-precisions= --no-kernel-timing --steps 20 --warmup 5"
for i in 1 2; do
  for side in skip noskip; do
    if [ $side = noskip ]; then export MRAGAN_NO_SKIP_STATS=1; else unset MRAGAN_NO_SKIP_STATS; fi
    step "b64 $side $i" 300 $B --full-out "$O/full_${side}_$i.json" > "$O/b64_${side}_$i.json" 2> "$O/b64_${side}_$i.err"
    python3 -c "import json; d=json.loads(open('$O/b64_${side}_$i.json').read().strip().splitlines()[-1]); print('64 $side $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
