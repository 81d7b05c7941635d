#!/bin/bash
# r04o: brickT one-plane variant (80-B halo rows, two blocks per CU, quarter-pass epilogue) —
# kernel tests, step parity subset, headline bench with top kernels
set -eo pipefail
TAG=${1:-r04o}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "three_tap or wgrad or stride2" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step stepp 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r6_s24_b1_pool1 or unet_s64" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
step bench 600 python3 bench.py --legs "128:1" --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("head", d["ms_per_step"], d.get("ms_per_step_median"))
for t in d.get("top_kernels", []):
    if "s2" in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["ms_per_step"], t["mean_us"], t["frac"])
for k, v in d.get("legs", {}).items():
    print("leg", k, v["ms_per_step"])
    for t in v.get("top_kernels", []):
        if "s2" in t["cls"]:
            print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["ms_per_step"], t["mean_us"], t["frac"])
PY
echo "[r04o] done"
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d "$O/p1" -o run -- python3 $R/tools/kbench.py --ops down1_wgrad,down2_wgrad --reps 5 --precision bf16 --N 4 > "$O/p1.log" 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/p2" -o run -- python3 $R/tools/kbench.py --ops down1_wgrad,down2_wgrad --reps 5 --precision bf16 --N 4 > "$O/p2.log" 2>&1 || true
python3 $R/tools/pmc_summary.py "$O" wgrad3s2 || true
