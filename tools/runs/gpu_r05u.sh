#!/bin/bash
# r05u: k4 s2 p1 weight gradients on the 4-tap even/odd-phase kernel — tests, kbench on / off,
# same-box step A/B (UNet leg, headline)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05u
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "four_tap or three_tap or wgrad" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
for v in on off; do
  if [ $v = off ]; then export MRAGAN_NO_W4S2=1; else unset MRAGAN_NO_W4S2; fi
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$v" -o run \
      -- python3 "$R/tools/kbench.py" --ops d2_wgrad,unet_up_wgrad --reps 20 --precision bf16 --N 4 > "$O/kb_$v.log" 2>&1 )
  python3 - "$O/kt_$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' in r['Name']:
        print(f"{sys.argv[2]:4s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
unset MRAGAN_NO_W4S2
step steptests 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -x -q -rf --tb=short --timeout 300 \
    --timeout-method thread -k "unet_s32 or unet_s64 or s64_b2" > "$O/step.log" 2>&1
tail -3 "$O/step.log"
BENCH_ARGS="--netG unet_custom --batch 1" bash tools/gpu_envab.sh r05u/unet 2 "-" "MRAGAN_NO_W4S2=1"
bash tools/gpu_envab.sh r05u/head 2 "-" "MRAGAN_NO_W4S2=1"
