#!/bin/bash
# r04n: res conv kernel durations under rocprofv3 (kernel time, not the Python call overhead) for
# the K-split brick variants vs the default choice, 64^3 N = 4 / 2
set -eo pipefail
TAG=${1:-r04n}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
source "$R/tools/gpu_step.sh"
for shp in "64 4" "64 2" "128 2"; do
  set -- $shp
  for v in 0 1 3; do
    if [ $v = 0 ]; then unset MRAGAN_BRICK_KS; else export MRAGAN_BRICK_KS=$v; fi
    d="$O/S$1_N$2_KS$v"
    step prof 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
      python3 "$R/tools/kbench.py" --ops res_fwd16,res_dgrad16s --reps 30 --precision bf16 --S $1 --N $2 > "$d.log" 2>&1
    echo "== S=$1 N=$2 KS=$v"
    f=$(find "$d" -name "run_kernel_stats.csv" | head -1)
    python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "brick" in n or "igemm" in n:
        print(f"   {n[:70]:70s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1000:8.2f} us")
PY
  done
done
unset MRAGAN_BRICK_KS
echo "[r04n] done"
