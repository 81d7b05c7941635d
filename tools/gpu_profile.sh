#!/bin/bash
# GPU-box profiling pass for one round: default bench line, rocprofv3 kernel-trace summary of
# the bench command, and the two PMC passes pricing HBM traffic of the dominant kernel.
#   bash tools/gpu_profile.sh r01
set -euo pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
echo "[gpu_profile] bench (default)"
timeout -k 10 600 python3 "$R/bench.py" > "$O/bench_default.json" 2> "$O/bench_default.err"
cat "$O/bench_default.json"
echo "[gpu_profile] kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/trace.log" 2>&1
echo "[gpu_profile] pmc FETCH_SIZE"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
    -- python3 "$R/tools/kbench.py" --ops res_fwd --reps 10 --precision bf16x3 > "$O/pmc_fetch.log" 2>&1
echo "[gpu_profile] pmc WRITE_SIZE"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run \
    -- python3 "$R/tools/kbench.py" --ops res_fwd --reps 10 --precision bf16x3 > "$O/pmc_write.log" 2>&1
# res conv fwd at 64^3 b2 (N=4 instances): padded input 4*18^3*128*4 + weights 27*128*128*4 + output 4*16^3*128*4
python3 "$R/tools/pmc_traffic.py" --fetch "$O/pmc_fetch" --write "$O/pmc_write" --kernel conv_brick \
    --key res_fwd:S64:N4:ngf32:bf16x3 --algorithmic-bytes 22102016 --out "$O/traffic.json"
echo "[gpu_profile] done"
