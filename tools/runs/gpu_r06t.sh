#!/bin/bash
# r06t: the stride-2 brick (G down1 / down2 forward, conv_brick_x3.hip S = 2) — kernel tests, bit-identity
# graph tests, step suites, per-variant rocprof kernel traces against the implicit GEMM, headline A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06t
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "stride2 or wgrad_short" > "$O/kern.log" 2>&1 || { tail -40 "$O/kern.log"; exit 1; }
tail -2 "$O/kern.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py -k "stride2 or headline" > "$O/graph.log" 2>&1 || { tail -40 "$O/graph.log"; exit 1; }
tail -2 "$O/graph.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_step_gpu.py -k "s64_b2 or s128 or s96" > "$O/steps.log" 2>&1 || { tail -40 "$O/steps.log"; exit 1; }
tail -2 "$O/steps.log"
cd /tmp && export TMPDIR=/tmp
KB="$R/tools/kbench.py --ops down1_fwd16,down1_fwd16s,down2_fwd16,down2_fwd16s --reps 20 --precision bf16"
for N in 4 2; do
  for V in 1 2 3 4; do
    MRAGAN_BRICK_S2_VAR=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_n${N}_v${V}" -o run \
        -- python3 $KB --N $N > "$O/kt_n${N}_v${V}.log" 2>&1
  done
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
for d in sorted(glob.glob(os.path.join(O, "kt_n*_v*"))):
    if not os.path.isdir(d):
        continue
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "igemm" in r["Name"] or "brick_x3" in r["Name"]:
                print(os.path.basename(d), r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us")
PY
cd "$R"
bash tools/gpu_envab.sh r06t/ab 3 "-" "MRAGAN_NO_BRICK_S2=1"
