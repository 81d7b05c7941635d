#!/bin/bash
# r04l: weight gradients on their own streams — graph bit-identity, step parity subset, DP test,
# and a same-box A/B of the headline step (MRAGAN_WGRAD_INLINE=1: in the lanes, as before)
set -eo pipefail
TAG=${1:-r04l}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step graph 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py tests/test_dp_gpu.py > "$O/graph.log" 2>&1
tail -2 "$O/graph.log"
step stepp 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r6_s24_b1_pool1 or unet_s64" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
run() {
  local v=$1; shift
  step bench_$v 300 env "$@" python3 bench.py --legs "" --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 \
    > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d.get('ms_per_step_median'))" "$O/bench_$v.json" $v
}
run wgs X=1
run inline MRAGAN_WGRAD_INLINE=1
run wgs2 X=1
run inline2 MRAGAN_WGRAD_INLINE=1
echo "[r04l] done"
