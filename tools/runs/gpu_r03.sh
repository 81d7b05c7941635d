#!/bin/bash
# Round-3 GPU pass: pytest -m gpu (optionally -k EXPR), the default bench line (64³ b2 + 128³ b1
# legs, alt precisions), logs under gpurun_out/TAG/.    bash tools/gpu_r03.sh TAG [KEXPR] [nobench]
set -eo pipefail
TAG=${1:-r03}
KEXPR=${2:-}
NOBENCH=${3:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
if [ "$KEXPR" != "none" ]; then
  step tests 900 python -u -m pytest tests -m gpu -v -rf --tb=short --timeout 300 --timeout-method thread \
      ${KEXPR:+-k "$KEXPR"} > "$O/pytest.log" 2>&1
  tail -4 "$O/pytest.log"
  grep -E "FAILED|ERROR" "$O/pytest.log" | head -30 || true
fi
if [ -z "$NOBENCH" ]; then
  step bench 700 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
  cut -c1-600 "$O/bench.json"
fi
echo "[r03] done"
