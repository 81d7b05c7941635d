#!/bin/bash
set -eo pipefail
TAG=${1:-r03h}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
for op in down1_fwd down2_fwd up1_fwd d2_fwd dfirst_dgrad; do
  bash tools/gpu_ab_env.sh "$TAG/$op" bf16 4 $op "- MRAGAN_IG_DEPTH1=1 MRAGAN_NO_TILE8=1"
done

python3 bench.py --alt-precisions '' --legs '' --no-cpu-baseline > gpurun_out/$TAG/bench_kt.json 2> gpurun_out/$TAG/bench_kt.err
python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], r['kernel_ms_per_step_serial'])" gpurun_out/$TAG/bench_kt.json
bash tools/gpu_variants.sh "$TAG/var" "--single-stream"
echo "[r03h] all done"
