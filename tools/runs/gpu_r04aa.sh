#!/bin/bash
# r04aa: wgrad3s2 K-half loop without per-step exec-mask branches; implicit GEMM incremental tap
# offsets — kernel tests, step subset, bench, PMC instruction mix of the stride-2 kernels
set -eo pipefail
TAG=${1:-r04aa}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "x3 or bf16x3 or stride2 or wgrad or op16 or transpose3d or all_paths or statistics or conv" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step stepp 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r6_s24 or r9_s32" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
step graph 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py > "$O/graph.log" 2>&1
tail -2 "$O/graph.log"
step bench 600 python3 bench.py --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("head", d["ms_per_step"], d.get("ms_per_step_median"), {k: v["ms_per_step"] for k, v in d["legs"].items()})
for t in d.get("top_kernels", []):
    if " s2 " in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["mean_us"], t["frac"])
PY
cd /tmp
KB="python3 $R/tools/kbench.py --ops down1_fwd16,down1_wgrad16,down2_fwd16,down2_wgrad16 --reps 5 --precision bf16 --N 4"
step mix 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY --output-format csv -d "$O/mix" -o run -- $KB > "$O/mix.log" 2>&1
step kt 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- $KB > "$O/kt.log" 2>&1
python3 $R/tools/pmc_summary.py "$O" igemm wgrad3s2 > "$O/pmc.txt" || true
cat "$O/pmc.txt"
python3 - "$O/kt/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:80])
PY
echo "[r04aa] done"
