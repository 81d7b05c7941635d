#!/bin/bash
# r04z: thin_n_tile8 with two channel quads per lane (the UNet outermost upconv, MFMA modes) —
# kernel tests, the UNet step cases, the UNet bench leg
set -eo pipefail
TAG=${1:-r04z}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "thin or transpose3d or all_paths" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step unet 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread tests/test_step_gpu.py -k "unet" \
  > "$O/unet.log" 2>&1
tail -2 "$O/unet.log"
step bench 600 python3 bench.py --legs "64:1:1:unet_custom:bf16" --alt-precisions "" --no-cpu-baseline --steps 30 \
  --warmup 5 > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
L = d["legs"]["64^3 b1 unet_custom"]
print("head", d["ms_per_step"], "unet", L["ms_per_step"], L["roofline"]["kernel"], L["roofline"]["launch_ms"])
for t in L.get("top_kernels", [])[:12]:
    print("  ", t["cls"], t["kernels"], t["launches_per_step"], t["mean_us"], t["frac"])
PY
echo "[r04z] done"
