#!/bin/bash
# r04ac: implicit GEMM with the parity classes fastest in the tile order (every XCD gets every
# class) — kernel tests, kbench of the transposed / stride-2 shapes, step subset, bench
set -eo pipefail
TAG=${1:-r04ac}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "x3 or bf16x3 or stride2 or transpose or all_paths or statistics or conv or shell or dgrad" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
bash tools/gpu_ab_env.sh "$TAG/ab4" bf16 4 up1_fwd,down1_fwd16,down2_fwd16,d2_fwd,dfirst_dgrad "-"
bash tools/gpu_ab_env.sh "$TAG/ab2" bf16 2 up1_fwd "-"
step stepp 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread tests/test_step_gpu.py \
  -k "r9_s64_b2 or r6_s24 or r9_s32 or unet" > "$O/step.log" 2>&1
tail -2 "$O/step.log"
step graph 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py > "$O/graph.log" 2>&1
tail -2 "$O/graph.log"
step bench 600 python3 bench.py --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("head", d["ms_per_step"], d.get("ms_per_step_median"), {k: v["ms_per_step"] for k, v in d["legs"].items()})
for t in d.get("top_kernels", []):
    if " s2 " in t["cls"]:
        print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["mean_us"], t["frac"])
PY
echo "[r04ac] done"
