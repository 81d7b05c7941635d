#!/bin/bash
# GPU-box pass: parity tests (selected by -k, or all), default bench line, a 2-rank gloo DP
# rehearsal on the one GPU.   bash tools/gpu_round.sh TAG ["pytest -k expr"]
set -euo pipefail
TAG=${1:-r02}
KEXPR=${2:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
echo "[round] pytest -m gpu ${KEXPR:+-k $KEXPR}"
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$KEXPR" > "$O/pytest.log" 2>&1 || { tail -60 "$O/pytest.log"; exit 1; }
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -60 "$O/pytest.log"; exit 1; }
fi
tail -3 "$O/pytest.log"
echo "[round] bench default"
timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -30 "$O/bench_default.err"; exit 1; }
cat "$O/bench_default.json"
echo "[round] bench dp2 rehearsal (gloo, same device)"
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --same-device --steps 5 --warmup 2 > "$O/bench_dp2.json" 2> "$O/bench_dp2.err" || { tail -30 "$O/bench_dp2.err"; exit 1; }
cat "$O/bench_dp2.json"
echo "[round] done"
