#!/bin/bash
# r06g: checkpoint at HEAD — the full -m gpu suite, smoke, the default bench line (driver form)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06g
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 900 python3 -u -m pytest tests -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
tail -2 "$O/smoke.log"
step bench 700 python3 bench.py --full-out "gpurun_out/r06g/bench_full.json" > "$O/bench.json" 2> "$O/bench.err"
cut -c1-400 "$O/bench.json"
