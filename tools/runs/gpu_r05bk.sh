#!/bin/bash
# 128³ step gates: bisect the split data gradient (MRAGAN_DGRAD_SPLIT=0) and conv2's split
# (MRAGAN_IN1_STATS_BIG=1)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bk}
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
T="python -u -m pytest tests/test_step_gpu.py -m gpu -q --timeout 300 --timeout-method thread -k s128_b1-bf16"
MRAGAN_DGRAD_SPLIT=0 step nosplit 300 $T > "$O/nosplit.log" 2>&1; tail -2 "$O/nosplit.log"
MRAGAN_IN1_STATS_BIG=1 step in1big 300 $T > "$O/in1big.log" 2>&1; tail -2 "$O/in1big.log"
MRAGAN_DGRAD_SPLIT=1 MRAGAN_IN1_STATS_BIG=1 step split_in1big 300 $T > "$O/split_in1big.log" 2>&1; tail -2 "$O/split_in1big.log"
