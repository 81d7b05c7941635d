#!/bin/bash
# One kernel's parity tests + its kbench timing under rocprofv3 (per-kernel durations).
#   bash tools/gpu_kcheck.sh TAG "PYTEST -k EXPR" "KBENCH OPS" [PREC] [N]
set -eo pipefail
TAG=$1; KEXPR=$2; OPS=$3; PREC=${4:-bf16}; KN=${5:-2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "$KEXPR" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
cd /tmp && export TMPDIR=/tmp
step ktrace 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run \
    -- python3 "$R/tools/kbench.py" --ops "$OPS" --reps 20 --precision "$PREC" --N "$KN" > "$O/ktrace.log" 2>&1
cat "$O/ktrace.log" | tail -8
F=$(find "$O/ktrace" -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$F" | head -12
