#!/bin/bash
# N = 4 res data gradient (18³ output, two rounds of K-split slots): the 8-wave brick (default)
# against the K-split variants forced (MRAGAN_BRICK_KS=1|2|3)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bp}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2 3; do
  ( if [ $v != 0 ]; then export MRAGAN_BRICK_KS=$v; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/v$v" -o run -- \
      python3 "$R/tools/kbench.py" --ops res_fwd16,res_dgrad16,res_dgrad16s --reps 20 --precision bf16 --N 4 > "$O/v$v.log" 2>&1 )
done
python3 /dev/stdin "$O" <<'PY'
import csv, glob, sys, os
for d in sorted(glob.glob(sys.argv[1] + '/v*/')):
    f = glob.glob(d + '/**/run_kernel_trace.csv', recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if 'conv_brick' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    out = []
    for i, op in enumerate(['fwd', 'dgrad', 'dgrad_s']):
        ch = rows[21 * i + 1: 21 * (i + 1)]
        out.append(f"{op} {sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in ch) / len(ch) / 1000:.1f} us "
                   f"[{ch[0]['Kernel_Name'].split('(')[0].replace('void mragan::', '')}]")
    print(os.path.basename(d.rstrip('/')), ' | '.join(out))
PY
