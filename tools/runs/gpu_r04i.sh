#!/bin/bash
# r04i: nc = 2 stem / head on the thin1 ring (two channels) and thinn (two outputs) kernels —
# kernel parity, the nc2 step cases, and the 96^3 nc2 fp16 configuration's step time
set -eo pipefail
TAG=${1:-r04i}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "thin or head_dgrad or in_stats_partials or all_paths_rounding or op16_brick" > "$O/kern.log" 2>&1
tail -3 "$O/kern.log"
step stepnc2 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_step_gpu.py -k "nc2" > "$O/step.log" 2>&1
tail -3 "$O/step.log"
step bench96 300 python3 bench.py --size 96 --batch 1 --nc 2 --precision fp16 --legs "" --alt-precisions "" \
  --no-cpu-baseline --steps 10 --warmup 3 > "$O/bench96.json" 2> "$O/bench96.err"
python3 - "$O/bench96.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("96 nc2 fp16", d["value"], d["ms_per_step"])
for t in d.get("top_kernels", [])[:14]:
    print("  ", t["cls"], t["kernels"], t["ms_per_step"], t["mean_us"], t["frac"])
PY
echo "[r04i] tests+bench done"
# headline kernel trace (graph-replayed steps; traced durations include inter-lane contention)
cd /tmp
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --legs "" --alt-precisions "" > "$O/trace.log" 2>&1
cd "$R"
python3 tools/prof_summary.py --steps 15 --top 60 "$O/trace/bench_kernel_trace.csv" > "$O/bench_kernels.md" || true
python3 tools/trace_lanes.py --last 5 "$O/trace/bench_kernel_trace.csv" > "$O/trace_lanes.md" || true
head -20 "$O/trace_lanes.md" || true
echo "[r04i] trace done"
