#!/bin/bash
# r04ae: timing-only igemm A/B (half the weight / input bytes dropped: MRAGAN_IG_TIMING=1/2), then the
# up1 plane path: plane-vs-fp32 step identity, step subset, bench
set -eo pipefail
TAG=${1:-r04ae}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
bash tools/gpu_ab_env.sh "$TAG/tm" bf16 4 up1_fwd,down1_fwd16,down2_fwd16,d2_fwd "- MRAGAN_IG_TIMING=1 MRAGAN_IG_TIMING=2"
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
for t in d.get("top_kernels", []):
    if "convT 128->64" in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["mean_us"], t["frac"])
PY
}
run pl X=1
run fp MRAGAN_NO_S2_PLANES=1
run pl2 X=1
echo "[r04ae] done"
