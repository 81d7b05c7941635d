#!/bin/bash
# r04d: PMC passes of the K-split brick variants (res fwd / dgrad, bf16, N = 4) + kernel A/B with the
# conflict-aware shape choice
set -eo pipefail
TAG=${1:-r04d}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
for v in 1; do
  MRAGAN_BRICK_KS=$v PREC=bf16 KN=4 step "pmc v$v" 400 bash tools/pmc_probe.sh $TAG/pmc_v$v res_fwd16,res_dgrad16
  python3 tools/pmc_summary.py "$O/pmc_v$v" brick > "$O/pmc_v$v.txt"; cat "$O/pmc_v$v.txt"
done
for N in 4 2; do
  step "kbench N$N" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$N" -o run -- python3 tools/kbench.py --ops res_fwd16,res_dgrad16 --reps 20 --precision bf16 --N $N > "$O/kbench_$N.log" 2>&1
  python3 - "$O/kt_$N" "N$N" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'brick' not in r['Kernel_Name']: continue
    d[(r['Kernel_Name'][:44], r['Grid_Size_X'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in d.items():
    v.sort(); print(sys.argv[2], k, len(v), 'median %.1f us' % v[len(v) // 2])
PY
done
echo "[r04d] done"
