#!/bin/bash
# r04y: UNet outermost upconv on thin_n_class8 (two quads per lane) in the MFMA modes; igemm BK 64
# (MRAGAN_IG_BK64) — kernel tests both ways, the UNet step cases, same-box bench A/B
set -eo pipefail
TAG=${1:-r04y}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
K="thin_class8 or bf16x3_fwd or bf16x3_wgrad or transpose3d or all_paths or stride2 or brick_in_stats or op16"
step kern 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "$K" \
  > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
step kern64 600 env MRAGAN_IG_BK64=1 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "$K" > "$O/kern64.log" 2>&1
tail -2 "$O/kern64.log"
step unet 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread tests/test_step_gpu.py -k "unet" \
  > "$O/unet.log" 2>&1
tail -2 "$O/unet.log"
run() {
  local v=$1; shift
  step bench_$v 600 env "$@" python3 bench.py --alt-precisions "" --no-cpu-baseline --steps 30 --warmup 5 \
    > "$O/bench_$v.json" 2> "$O/bench_$v.err"
  python3 - "$O/bench_$v.json" $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "head", d["ms_per_step"], d.get("ms_per_step_median"), {k: v["ms_per_step"] for k, v in d["legs"].items()})
for t in d.get("top_kernels", []):
    if "conv_igemm" in t["kernels"]:
        print("  ", t["cls"], t["launches_per_step"], t["mean_us"], t["frac"])
PY
}
run base X=1
run bk64 MRAGAN_IG_BK64=1
run base2 X=1
run bk642 MRAGAN_IG_BK64=1
echo "[r04y] done"
