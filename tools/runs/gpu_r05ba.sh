#!/bin/bash
# Res-block conv kernels under env variants (ticket finalize, K-split on/off, big-grid K-split):
# rocprofv3 kernel-trace averages of tools/kbench.py at the 64³ b2 (N = 4, 2) and 128³ b1 (N = 2, 1)
# res-level shapes.   bash tools/runs/gpu_r05ba.sh TAG
set -eo pipefail
TAG=${1:-r05ba}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
OPS=res_fwd16,res_dgrad16,res_dgrad16s,res_wgrad16
run() {   # name S N env...
  local name=$1 S=$2 N=$3; shift 3
  echo "[run] $name S=$S N=$N $*" >&2
  ( export "$@" 2>/dev/null; timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o run -- \
      python3 "$R/tools/kbench.py" --ops $OPS --reps 20 --precision bf16 --S "$S" --N "$N" > "$O/$name.log" 2>&1 )
  python3 - "$O/$name" "$name" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' not in r['Name']:
        continue
    print(f"{sys.argv[2]:>18s} {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
}
for SN in "64 4" "64 2" "128 2" "128 1"; do
  set -- $SN; S=$1; N=$2
  run "s${S}n${N}_def" $S $N MRAGAN_DUMMY=1
  run "s${S}n${N}_notick" $S $N MRAGAN_NO_IN_TICKETS=1
  run "s${S}n${N}_noks" $S $N MRAGAN_BRICK_KS=0
  run "s${S}n${N}_nobig" $S $N MRAGAN_KS_BIG=0
done 2>&1 | tee "$O/summary.txt"
