#!/bin/bash
# Same-box step A/B of an environment switch: bench.py (no CPU leg) alternately with VAR=1 and
# without, twice each.   bash tools/gpu_bench_ab.sh TAG VAR
set -eo pipefail
TAG=$1; VAR=$2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
for i in 1 2; do
  for side in off on; do
    if [ $side = on ]; then export $VAR=1; else unset $VAR; fi
    step "bench $side $i" 300 python3 bench.py --no-cpu-baseline --alt-precisions "" > "$O/bench_${side}_$i.json" 2> "$O/bench_${side}_$i.err"
    python3 -c "import json; d=json.load(open('$O/bench_${side}_$i.json')); print('$VAR=$side run $i', d['value'], d['ms_per_step'], d['ms_per_step_median'])"
  done
done
