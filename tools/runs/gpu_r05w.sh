#!/bin/bash
# r05w: brickT with 1 / 2 / 4 waves per block — tests, kbench per NW, step A/B (UNet, headline)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05w
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "brickT or transpose or dgrad or all_paths or op16" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
for nw in 0 4 2 1; do
  if [ $nw = 0 ]; then unset MRAGAN_BRICKT_NW; else export MRAGAN_BRICKT_NW=$nw; fi
  for n in 1 2 4; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${nw}_$n" -o run \
        -- python3 "$R/tools/kbench.py" --ops unet_ct,up2_fwd --reps 20 --precision bf16 --N $n > "$O/kb_${nw}_$n.log" 2>&1 )
    python3 - "$O/kt_${nw}_$n" "NW=$nw N=$n" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'brickT_x3' in r['Name']:
        print(f"{sys.argv[2]:10s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
  done
done
unset MRAGAN_BRICKT_NW
step steptests 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -x -q -rf --tb=short --timeout 300 \
    --timeout-method thread -k "unet_s32 or unet_s64 or s64_b2" > "$O/step.log" 2>&1
tail -3 "$O/step.log"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r05w/unet 2 "-" "MRAGAN_BRICKT_NW=4"
bash tools/gpu_envab.sh r05w/head 2 "-" "MRAGAN_BRICKT_NW=4"
