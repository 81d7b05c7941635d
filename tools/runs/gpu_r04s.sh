#!/bin/bash
# r04s: 16-bit operand planes for G down1 / down2 (ABI 14) — kernel tests, the plane-vs-fp32 step
# A/B, the reduced-precision step subset, same-box bench A/B (MRAGAN_NO_S2_PLANES) + kernel trace
set -eo pipefail
TAG=${1:-r04s}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "stride2 or op16 or wgrad_s2" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step planes 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py \
  -k "stride2_planes or bf16" > "$O/planes.log" 2>&1
tail -2 "$O/planes.log"
step stepp 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r9_s96 or r9_s128" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
run() {
  local v=$1; shift
  step bench_$v 600 env "$@" python3 bench.py --legs "128:1" --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 \
    > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 - "$O/bench_$v.json" $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "head", d["ms_per_step"], d.get("ms_per_step_median"), "128:", d["legs"]["128^3 b1"]["ms_per_step"])
for t in d.get("top_kernels", []):
    if " s2 " in t["cls"] or "k3 s2" in t["cls"] or "instnorm_fwd C32" in t["cls"] or "instnorm_fwd C64" in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["ms_per_step"], t["mean_us"], t["frac"])
PY
}
run pl X=1
run fp MRAGAN_NO_S2_PLANES=1
run pl2 X=1
echo "[r04s] done"
