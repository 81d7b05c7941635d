#!/bin/bash
# r04af: same-box A/B of HEAD's library against the r04final2 commit's (ablib/, MRAGAN_HIP_LIB),
# headline + bf16x3, alternating
set -eo pipefail
TAG=${1:-r04af}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
run() {
  local v=$1; shift
  step bench_$v 600 env "$@" python3 bench.py --legs "" --alt-precisions "bf16x3" --no-cpu-baseline --steps 30 --warmup 5 \
    > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 - "$O/bench_$v.json" $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "head", d["ms_per_step"], d.get("ms_per_step_median"), "bf16x3", d["alt_precisions"]["bf16x3"]["ms_per_step"])
PY
}
run head X=1
run old MRAGAN_HIP_LIB=$R/ablib/libmragan_hip_6b93.so
run head2 X=1
run old2 MRAGAN_HIP_LIB=$R/ablib/libmragan_hip_6b93.so
echo "[r04af] done"
