#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05aa
mkdir -p "$O"
for v in 0 1; do
  if [ $v = 1 ]; then export MRAGAN_DGRAD_SPLIT=1; else unset MRAGAN_DGRAD_SPLIT; fi
  for S in 64 128; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${v}_$S" -o run \
      -- python3 "$R/tools/kbench.py" --ops res_dgrad --reps 10 --precision bf16 --N 2 --S $S > "$O/kb_$v.log" 2>&1 )
  python3 - "$O/kt_${v}_$S" "SPLIT=$v S=$S" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' in r['Name'] and 'pack' not in r['Name']:
        print(f"{sys.argv[2]:14s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
  done
done
