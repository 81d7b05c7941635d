#!/bin/bash
# wgrad_reduce: 32-gn × all-taps rows (default) vs the 64 × 4 tiles (MRAGAN_RED_TILES=1) — weight
# gradient kernel tests, kbench kernel-trace means, then the 64³ step alternating
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bm}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step ktests 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad" > "$O/ktests.log" 2>&1
tail -2 "$O/ktests.log"
grep -q "failed" "$O/ktests.log" && exit 1
cd /tmp && export TMPDIR=/tmp
for side in rows tiles; do
  for N in 4 2; do
    if [ $side = tiles ]; then export MRAGAN_RED_TILES=1; else unset MRAGAN_RED_TILES; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${side}_n$N" -o run -- \
      python3 "$R/tools/kbench.py" --ops res_wgrad16,d2_wgrad,unet_up_wgrad --reps 20 --precision bf16 --N $N > "$O/${side}_n$N.log" 2>&1
    python3 - "$O/${side}_n$N" "${side} N=$N" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'reduce' in r['Name'] or 'wgrad' in r['Name']:
        print(f"{sys.argv[2]:>12s} {float(r['AverageNs'])/1000:8.1f} us x{r['Calls']:>4} {r['Name'][:70]}")
PY
  done
done
cd "$R"
B="python3 bench.py --legs= --no-cpu-baseline --alt-precisions= --no-kernel-timing --steps 20 --warmup 5"
for i in 1 2; do
  for side in rows tiles; do
    if [ $side = tiles ]; then export MRAGAN_RED_TILES=1; else unset MRAGAN_RED_TILES; fi
    step "b64 $side $i" 300 $B --full-out "$O/full_${side}_$i.json" > "$O/b64_${side}_$i.json" 2> "$O/b64_${side}_$i.err"
    python3 -c "import json; d=json.loads(open('$O/b64_${side}_$i.json').read().strip().splitlines()[-1]); print('64 $side $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
