#!/bin/bash
# Round-end style GPU pass: all -m gpu tests, smoke, the default bench line, a clean kernel trace
# of the headline workload (no per-class timing: the trace holds only the W+K steps) and the
# FETCH_SIZE / WRITE_SIZE passes of the res-block kernels.   bash tools/gpu_r03_full.sh TAG [notests]
set -eo pipefail
TAG=${1:-r03full}
NOTESTS=${2:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
if [ -z "$NOTESTS" ]; then
  step tests 900 python -u -m pytest tests -m gpu -v -rf --tb=short --timeout 300 --timeout-method thread \
      > "$O/pytest.log" 2>&1
  tail -3 "$O/pytest.log"
  grep -E "FAILED|ERROR" "$O/pytest.log" | head -20 || true
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -2 "$O/smoke.log"
fi
step bench 700 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
cut -c1-400 "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-kernel-timing --alt-precisions '' --legs '' --no-cpu-baseline \
    > "$O/trace.log" 2>&1
KB="$R/tools/kbench.py --ops res_wgrad,res_dgrad,res_fwd --reps 10 --precision bf16"
step fetch 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- python3 $KB > "$O/fetch.log" 2>&1
step write 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- python3 $KB > "$O/write.log" 2>&1
echo "[full] done"
