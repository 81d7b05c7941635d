#!/bin/bash
# r04a: K-split brick (conv_brick_ks.hip) — kernel parity tests, same-box kernel A/B against the
# r03 brick (MRAGAN_BRICK_KS=0), short bf16 step A/B.
set -eo pipefail
TAG=${1:-r04a}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kt 600 python -u -m pytest tests/test_kernels_gpu.py -q -rf --tb=short --timeout 300 --timeout-method thread -k "op16 or brick or backward_statistics or in_stats" > "$O/kt.log" 2>&1
grep -E "passed|failed" "$O/kt.log" | tail -1; grep -E "^FAILED" "$O/kt.log" | head -20 || true
grep -q " failed" "$O/kt.log" && { echo "kernel tests failed"; exit 1; }
for N in 4 2; do
for side in off on; do
  if [ $side = off ]; then export MRAGAN_BRICK_KS=0; else unset MRAGAN_BRICK_KS; fi
  step "kbench $side N$N" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${side}_$N" -o run -- python3 tools/kbench.py --ops res_fwd16,res_dgrad16 --reps 20 --precision bf16 --N $N > "$O/kbench_${side}_$N.log" 2>&1
  python3 - "$O/kt_${side}_$N" "$side N$N" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r['Name'].startswith('void at::') or 'rocclr' in r['Name']:
        continue
    print(f"{sys.argv[2]:7s} {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
done
unset MRAGAN_BRICK_KS
for side in on off on; do
  if [ $side = off ]; then export MRAGAN_BRICK_KS=0; else unset MRAGAN_BRICK_KS; fi
  step "bench $side" 300 python3 bench.py --steps 20 --warmup 5 --alt-precisions '' --legs '' --no-cpu-baseline --no-kernel-timing > "$O/bench_$side.json" 2> "$O/bench_$side.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['ms_per_step_median'])" "$O/bench_$side.json" "$side"
done
echo "[r04a] done"
