#!/bin/bash
# Quick GPU iteration pass: selected parity tests, kernel microbench trace, short bench.
#   bash tools/gpu_quick.sh TAG "pytest -k expr" "kbench ops"
set -euo pipefail
TAG=${1:-quick}
KEXPR=${2:-brick}
KOPS=${3:-res_fwd,res_dgrad,res_wgrad}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
echo "[quick] tests -k $KEXPR"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
cd /tmp && export TMPDIR=/tmp
echo "[quick] kbench trace"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/tools/kbench.py" --ops "$KOPS" --reps 10 --precision bf16x3 > "$O/kbench.log" 2>&1
grep "us/call" "$O/kbench.log" || true
echo "[quick] bench"
timeout -k 10 300 python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err"
grep '^{' "$O/bench.json"
