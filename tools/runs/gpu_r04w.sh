#!/bin/bash
# r04w: in-launch InstanceNorm finalize (ABI 15, ticket counters in the K-split brick) — kernel
# tests, graph-vs-eager identity, the reduced-precision step subset, then a same-box A/B of the
# headline (MRAGAN_NO_IN_TICKETS: the finalize launches; MRAGAN_IN_FIN_LDS: r04's finalize combine)
set -eo pipefail
TAG=${1:-r04w}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "finalize or op16 or instnorm or statistics" -rs > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step graph 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py \
  > "$O/graph.log" 2>&1
tail -2 "$O/graph.log"
step stepp 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "bf16 or fp16" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
run() {
  local v=$1; shift
  step bench_$v 600 env "$@" python3 bench.py --legs "128:1" --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 \
    > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 - "$O/bench_$v.json" $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "head", d["ms_per_step"], d.get("ms_per_step_median"), "128:", d["legs"]["128^3 b1"]["ms_per_step"])
PY
}
run tk X=1
run nt MRAGAN_NO_IN_TICKETS=1
run lds MRAGAN_NO_IN_TICKETS=1 MRAGAN_IN_FIN_LDS=1
run tk2 X=1
run nt2 MRAGAN_NO_IN_TICKETS=1
echo "[r04w] done"
