#!/bin/bash
# r04k: fused-finalize A/B variants of the headline step (same box)
set -eo pipefail
TAG=${1:-r04k}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
run() {
  local v=$1; shift
  step bench_$v 300 env "$@" python3 bench.py --legs "" --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 \
    > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d.get('ms_per_step_median'))" "$O/bench_$v.json" $v
}
run base X=1
run f_small MRAGAN_IN_FUSED=1 MRAGAN_IN_FUSED_CAPSTATS=0 MRAGAN_IN_FUSED_CAP=131072 MRAGAN_IN_FUSED_MAXMB=8
run f_small64 MRAGAN_IN_FUSED=1 MRAGAN_IN_FUSED_CAPSTATS=0 MRAGAN_IN_FUSED_CAP=65536 MRAGAN_IN_FUSED_MAXMB=8
run f_all_nocap MRAGAN_IN_FUSED=1 MRAGAN_IN_FUSED_CAPSTATS=0 MRAGAN_IN_FUSED_CAP=131072
run base2 X=1
python3 - "$O/bench_f_small.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for t in d.get("top_kernels", []):
    if "instnorm" in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["ms_per_step"], t["mean_us"], t["frac"])
PY
echo "[r04k] done"
