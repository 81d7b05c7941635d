#!/bin/bash
# r04c: K-split brick variants (two per CU / one per CU TN1 / TN2) vs the r03 brick: parity tests,
# phase stamps, kernel A/B (rocprof), short bf16 step A/B
set -eo pipefail
TAG=${1:-r04c}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kt 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --tb=short --timeout 300 --timeout-method thread -k "op16 or brick or backward_statistics or in_stats or test_conv" > "$O/kt.log" 2>&1
tail -1 "$O/kt.log"; grep -E "^FAILED|Error" "$O/kt.log" | head -5 || true
grep -q " failed" "$O/kt.log" && { echo "kernel tests failed"; exit 1; }
for v in 1 2 3; do
  MRAGAN_BRICK_KS=$v step "stamps v$v" 200 python3 tools/diag_ks.py bf16 > "$O/stamps_v$v.txt" 2>&1
  echo "v$v"; grep -v amdgpu.ids "$O/stamps_v$v.txt"
done
for N in 4 2; do
for v in 0 1 2 3; do
  export MRAGAN_BRICK_KS=$v
  step "kbench v$v N$N" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${v}_$N" -o run -- python3 tools/kbench.py --ops res_fwd16,res_dgrad16 --reps 20 --precision bf16 --N $N > "$O/kbench_${v}_$N.log" 2>&1
  python3 - "$O/kt_${v}_$N" "v$v N$N" <<'PY'
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
done
unset MRAGAN_BRICK_KS
for side in on off on off; do
  if [ $side = off ]; then export MRAGAN_BRICK_KS=0; else unset MRAGAN_BRICK_KS; fi
  step "bench $side" 300 python3 bench.py --steps 20 --warmup 5 --alt-precisions '' --legs '' --no-cpu-baseline --no-kernel-timing > "$O/bench_$side.json" 2> "$O/bench_$side.err"
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['ms_per_step_median'])" "$O/bench_$side.json" "$side"
done
echo "[r04c] done"
