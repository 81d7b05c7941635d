#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02f
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 900 python -u -m pytest tests -m gpu -q -rA --tb=short --timeout 300 --timeout-method thread -k "step_gpu or dp_two or graph_step" -s > "$O/pytest.log" 2>&1
grep -E "passed|failed|FAILED|whole-net|stepped differently|dp vs single|loss rel err" "$O/pytest.log" | tail -150
for p in bf16x3 bf16 fp16; do
  step "bench $p" 300 python3 bench.py --precision $p --no-cpu-baseline --steps 10 --warmup 3 > "$O/bench_$p.json" 2> "$O/bench_$p.err"
  cat "$O/bench_$p.json"
done
