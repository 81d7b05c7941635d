#!/bin/bash
# r04j: InstanceNorm finalize fused into the apply kernels — norm kernel tests, graph bit-identity,
# step parity subset, and a same-box A/B of the headline step (MRAGAN_IN_UNFUSED=1: separate launches)
set -eo pipefail
TAG=${1:-r04j}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "instnorm or in_stats or statistics or op16 or rpad" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step graph 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py > "$O/graph.log" 2>&1
tail -2 "$O/graph.log"
step stepp 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r6_s24_b1_pool1 or nc2_lsgan" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
for v in fused unfused fused2; do
  if [ $v = unfused ]; then export MRAGAN_IN_UNFUSED=1; else unset MRAGAN_IN_UNFUSED; fi
  step bench_$v 300 python3 bench.py --legs "" --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 \
    > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d.get('ms_per_step_median'))" "$O/bench_$v.json" $v
done
unset MRAGAN_IN_UNFUSED
python3 - "$O/bench_fused.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for t in d.get("top_kernels", []):
    if "instnorm" in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["ms_per_step"], t["mean_us"], t["frac"])
PY
echo "[r04j] done"
