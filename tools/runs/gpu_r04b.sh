#!/bin/bash
# r04b: K-split brick phase stamps + kernel A/B
set -eo pipefail
TAG=${1:-r04b}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kt 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --tb=short --timeout 300 --timeout-method thread -k "op16_brick or op16_dgrad or in_stats_partials or test_conv" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"
step stamps 200 python3 tools/diag_ks.py bf16 > "$O/stamps.txt" 2>&1
cat "$O/stamps.txt"
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
echo "[r04b] done"
