#!/bin/bash
# split vs whole-grid ResnetBlock data gradient at the 96³ configuration's 24³ level (fp16) and 2 × 28³
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bj}
mkdir -p "$O"
cd "$R"
MRAGAN_DGRAD_SPLIT=0 timeout -k 10 120 python3 tools/probes/split_dgrad_probe.py fp16 2x24,4x24,2x28 2>&1 | tee "$O/whole.txt"
MRAGAN_DGRAD_SPLIT=1 timeout -k 10 120 python3 tools/probes/split_dgrad_probe.py fp16 2x24,4x24,2x28 2>&1 | tee "$O/split.txt"
