#!/bin/bash
# Headline-workload step time under schedule variants (no per-class timing, no CPU leg), one
# bench.py run per variant, same box:   bash tools/gpu_variants.sh TAG "ARGS1" "ARGS2" ...
set -eo pipefail
TAG=${1:-var}
shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
i=0
for v in "$@"; do
  i=$((i + 1))
  echo "[var $i] $v" | tee -a "$O/variants.txt"
  step "v$i" 240 python3 bench.py --alt-precisions '' --legs '' --no-cpu-baseline --no-kernel-timing $v \
      > "$O/v$i.json" 2> "$O/v$i.err"
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], r['ms_per_step_median'])" "$O/v$i.json" | tee -a "$O/variants.txt"
done
echo "[variants] done"
