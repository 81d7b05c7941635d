#!/bin/bash
# r04v: InstanceNorm finalize with a wave butterfly (no 64-step LDS combine) — IN kernel tests, the
# reduced-precision step subset, the headline bench, and a kernel trace of the bench
set -eo pipefail
TAG=${1:-r04v}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "instnorm or in_stats or partials or statistics" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step stepp 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r6_s24" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
step bench 600 python3 bench.py --legs "128:1" --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 \
  > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("head", d["ms_per_step"], d.get("ms_per_step_median"), "128:", d["legs"]["128^3 b1"]["ms_per_step"])
PY
cd /tmp
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --legs "" --alt-precisions "" > "$O/trace.log" 2>&1
python3 - "$O/trace/bench_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "in_" in r["Name"] and "mragan::" in r["Name"]:
        print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:70])
PY
echo "[r04v] done"
