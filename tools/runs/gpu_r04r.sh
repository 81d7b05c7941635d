#!/bin/bash
# r04r: wgrad3 64-row waves (128x64 operand-plane tiles on 4 waves) — kernel tests, step subset,
# same-box A/B of the headline and the 128^3 leg (MRAGAN_W3_WM=1: the 8-wave tiles)
set -eo pipefail
TAG=${1:-r04r}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "op16 or wgrad3 or wgrad" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step stepp 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r9_s96" > "$O/step.log" 2>&1
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
    if "wgrad 128x128" in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["ms_per_step"], t["mean_us"], t["frac"])
for t in d["legs"]["128^3 b1"].get("top_kernels", []):
    if "wgrad 128x128" in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["ms_per_step"], t["mean_us"], t["frac"])
PY
}
run wm2 X=1
run wm1 MRAGAN_W3_WM=1
run wm2b X=1
echo "[r04r] done"
