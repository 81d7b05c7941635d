#!/bin/bash
# A/B bench variants: bash tools/gpu_ab.sh TAG "ENV=.. args" "ENV=.. args" ...   (one bench per variant)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
i=0
for v in "$@"; do
  i=$((i+1))
  echo "[ab] $i: $v"
  envs=(); args=()
  for t in $v; do if [[ "$t" == -* ]]; then args+=("$t"); else envs+=("$t"); fi; done
  env "${envs[@]}" timeout -k 10 300 python3 bench.py --no-cpu-baseline --alt-precisions "" "${args[@]}" > "$O/v$i.json" 2> "$O/v$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "[ab] variant $i rc $rc — stopping"; tail -5 "$O/v$i.err"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('   ', d['value'], d['ms_per_step'], d['ms_per_step_median'])" "$O/v$i.json"
done
