#!/bin/bash
# Same-box A/B of env settings on the quick headline bench (no legs / alt precisions / CPU baseline /
# kernel timing), alternating, ROUNDS rounds:  bash tools/gpu_envab.sh TAG ROUNDS "ENV1" "ENV2" ...
# ("-" = no extra env); extra bench.py arguments in $BENCH_ARGS (e.g. "--netG unet_custom --batch 1")
set -eo pipefail
TAG=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --legs '' --alt-precisions '' --no-cpu-baseline \
        --no-kernel-timing --full-out '' $BENCH_ARGS > "$O/ab_${r}_${i}.json" 2> "$O/ab_${r}_${i}.err"
    python3 -c "import json,sys; d=json.load(open('$O/ab_${r}_${i}.json')); print('round $r', repr('$e'), d['ms_per_step'], d['ms_per_step_median'])"
  done
done
