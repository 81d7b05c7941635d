#!/bin/bash
# r05y: brickT for 64-output-channel transposed convs (32-channel groups) — tests, kbench on / off,
# headline A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05y
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "brickT or transpose or dgrad or all_paths or op16" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
for v in 1 0; do
  export MRAGAN_BRICKT_WIDE=$v
  for n in 2 4; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${v}_$n" -o run \
        -- python3 "$R/tools/kbench.py" --ops up1_fwd --reps 20 --precision bf16 --N $n > "$O/kb_${v}_$n.log" 2>&1 )
    python3 - "$O/kt_${v}_$n" "WIDE=$v N=$n" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' in r['Name'] and 'pack' not in r['Name']:
        print(f"{sys.argv[2]:10s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
  done
done
unset MRAGAN_BRICKT_WIDE
step steptests 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -x -q -rf --tb=short --timeout 300 \
    --timeout-method thread -k "s64_b2 or s32_b1 or s128" > "$O/step.log" 2>&1
tail -3 "$O/step.log"
bash tools/gpu_envab.sh r05y/head 2 "-" "MRAGAN_BRICKT_WIDE=0"
