#!/bin/bash
# igemm tile-config sweep on the stride-2 / PatchGAN convs (MRAGAN_IGEMM_CFG was an A/B switch
# while the plan rule was chosen; with it removed every run times the shipped plan).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
for c in ${CFGS:--1 0 1 2 3 4}; do
  export MRAGAN_IGEMM_CFG=$c
  step "cfg $c" 200 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/igcfg/kt_$c" -o run -- python3 tools/kbench.py --ops down1_fwd,down2_fwd,up1_fwd,d2_fwd --reps 10 --precision bf16x3 > "gpurun_out/igcfg/kb_$c.log" 2>&1
  python3 - "gpurun_out/igcfg/kt_$c" "$c" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
d = defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if 'igemm' in n or 'splitk' in n:
        d[(n.split('(')[0].replace('void mragan::', '')[:45], r['Grid_Size_X'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k in sorted(d): print('cfg', sys.argv[2], k, round(sum(d[k]) / len(d[k]), 1), len(d[k]))
PY
done
