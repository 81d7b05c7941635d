#!/bin/bash
# Same-box step A/B over environment settings: "-" = default; each other word VAR=VALUE[;VAR=VALUE].
#   bash tools/gpu_stepenv_ab.sh TAG "- MRAGAN_W3_BLOCKS=128 ..."
set -eo pipefail
TAG=$1; SETS=$2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
i=0
for e in $SETS; do
  i=$((i + 1))
  envs=()
  if [ "$e" != "-" ]; then IFS=';' read -ra envs <<< "$e"; envs=(env "${envs[@]}"); fi
  step "s$i" 240 "${envs[@]}" python3 bench.py --alt-precisions '' --legs '' --no-cpu-baseline --no-kernel-timing \
      > "$O/s$i.json" 2> "$O/s$i.err"
  python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(f\"{sys.argv[2]:>40s} {r['value']:8.2f} p/s {r['ms_per_step']:7.3f} ms (median {r['ms_per_step_median']:.3f})\")" "$O/s$i.json" "$e" | tee -a "$O/summary.txt"
done
echo "[stepenv] done"
