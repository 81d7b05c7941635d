#!/bin/bash
# r06c: UNet step suites after the pairing kwargs fix; the wgrad3 block budget re-tuned for the
# paired [6×16³] launch (same box, alternating); the default bench line (legs, H2D, phases)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06c
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step steps 600 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread \
    -k "unet" > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
bash tools/gpu_envab.sh r06c/ab 2 "-" "MRAGAN_W3_BLOCKS=128" "MRAGAN_W3_BLOCKS=256" "MRAGAN_W3_BLOCKS=96"
step bench 600 python3 bench.py --full-out "gpurun_out/r06c/bench_full.json" > "$O/bench.json" 2> "$O/bench.err"
cut -c1-300 "$O/bench.json"
