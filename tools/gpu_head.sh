#!/bin/bash
# One GPU-box pass at HEAD: full -m gpu suite, default bench line, rocprofv3 kernel trace of the
# bench command, and FETCH_SIZE / WRITE_SIZE passes for the bench's dominant launch class
# (res-block data gradient, conv_brick_x3 [4x16^3] -> 18^3), merged into profiles-ready files.
#   bash tools/gpu_head.sh TAG [skip-tests]
set -euo pipefail
TAG=${1:-r02h}
SKIP=${2:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -z "$SKIP" ]; then
  echo "[head] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -60 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
echo "[head] smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
echo "[head] bench default"
timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -30 "$O/bench_default.err"; exit 1; }
cat "$O/bench_default.json"
echo "[head] bench dp2 rehearsal (gloo, same device)"
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --same-device --steps 5 --warmup 2 --no-cpu-baseline \
    --alt-precisions "" > "$O/bench_dp2.json" 2> "$O/bench_dp2.err" || { tail -30 "$O/bench_dp2.err"; exit 1; }
grep '^{' "$O/bench_dp2.json" | cut -c1-200
cd /tmp && export TMPDIR=/tmp
echo "[head] kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --alt-precisions "" > "$O/trace.log" 2>&1
echo "[head] pmc FETCH_SIZE / WRITE_SIZE (res dgrad)"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
    -- python3 "$R/tools/kbench.py" --ops res_dgrad --reps 10 --precision bf16x3 > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run \
    -- python3 "$R/tools/kbench.py" --ops res_dgrad --reps 10 --precision bf16x3 > "$O/pmc_write.log" 2>&1
# dgrad at 64^3 b2 (N=4): dy 4*16^3*128*4 + weights 27*128*128*4 + dx 4*18^3*128*4 bytes
python3 "$R/tools/pmc_traffic.py" --fetch "$O/pmc_fetch" --write "$O/pmc_write" --kernel conv_brick \
    --key "conv_brick_x3|convT 128->128 k3 s1 [4x16x16x16]" --algorithmic-bytes 22102016 --out "$O/traffic.json" \
    --source "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tools/kbench.py --ops res_dgrad (64^3 b2 shape), profiles/$TAG"
echo "[head] done"
