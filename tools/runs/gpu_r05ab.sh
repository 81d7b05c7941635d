#!/bin/bash
# r05ab: thin1r forward with two blocks per CU (compact LDS), 8-voxel wgrad3s2 segments — tests,
# kbench TW 2 vs 1, step A/B
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05ab
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "thin1 or head_dgrad or k7_planes or stem or wgrad_s2 or bf16x3_wgrad" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
for tw in 2 1; do
  export MRAGAN_THIN1_TW=$tw
  for S in 64 128; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_${tw}_$S" -o run \
        -- python3 "$R/tools/kbench.py" --ops stem_fwd_st,stem_fwd,head_dgrad_st --reps 10 --precision bf16 --N 2 --S $S > "$O/kb_${tw}_$S.log" 2>&1 )
    python3 - "$O/kt_${tw}_$S" "TW=$tw S=$S" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'thin1r' in r['Name']:
        print(f"{sys.argv[2]:12s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
  done
done
unset MRAGAN_THIN1_TW
step steptests 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -x -q -rf --tb=short --timeout 300 \
    --timeout-method thread -k "s64_b2 or s32_b1 or s128" > "$O/step.log" 2>&1
tail -3 "$O/step.log"
bash tools/gpu_envab.sh r05ab/head 2 "-" "MRAGAN_THIN1_TW=1" "MRAGAN_NO_W3S2_SW8=1"
BENCH_ARGS="--size 128 --batch 1" bash tools/gpu_envab.sh r05ab/l128 2 "-" "MRAGAN_THIN1_TW=1" "MRAGAN_KS_BIG=0"
BENCH_ARGS="--size 64 --batch 1 --netG unet_custom" bash tools/gpu_envab.sh r05ab/unet 2 "-" "MRAGAN_NO_W3S2_SW8=1" "MRAGAN_WGRAD_NO_DIRECT=1"
bash tools/gpu_trace_leg.sh r05ab/unet_trace --size 64 --batch 1 --netG unet_custom
