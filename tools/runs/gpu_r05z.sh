#!/bin/bash
# r05z: res-block kernels at the 128³ leg's size (32³ res grid, N = 2): brick_x3 vs forced K-split,
# plain and with backward statistics; headline step A/B of forcing the K-split brick
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05z
mkdir -p "$O"
for v in 0 1; do
  if [ $v = 1 ]; then export MRAGAN_BRICK_KS=1; else unset MRAGAN_BRICK_KS; fi
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$v" -o run \
      -- python3 "$R/tools/kbench.py" --ops res_fwd16,res_dgrad16,res_dgrad16s,res_wgrad16 --reps 10 --precision bf16 --N 2 --S 128 > "$O/kb_$v.log" 2>&1 )
  python3 - "$O/kt_$v" "KS=$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' in r['Name'] and 'pack' not in r['Name']:
        print(f"{sys.argv[2]:6s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
unset MRAGAN_BRICK_KS
cd "$R"
bash tools/gpu_envab.sh r05z/head 2 "-" "MRAGAN_BRICK_KS=1"
