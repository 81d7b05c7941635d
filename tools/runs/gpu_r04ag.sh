#!/bin/bash
# r04ag: up1 / up2 backward on planes (ABI 16) — kernel tests, plane-vs-fp32 step identity, the
# reduced-precision step subset, same-box bench A/B (MRAGAN_NO_S2_PLANES)
set -eo pipefail
TAG=${1:-r04ag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "op16 or stride2" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step planes 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py > "$O/planes.log" 2>&1
tail -2 "$O/planes.log"
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
run pl X=1
run fp MRAGAN_NO_S2_PLANES=1
run pl2 X=1
run fp2 MRAGAN_NO_S2_PLANES=1
echo "[r04ag] done"
