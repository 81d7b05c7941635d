#!/bin/bash
# interior + shell data gradient on operand planes (MRAGAN_DGRAD_SPLIT=1) vs the whole-grid brick:
# fp64 check + HIP-event times (tools/probes/split_dgrad_probe.py), both modes
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bb}
mkdir -p "$O"
cd "$R"
timeout -k 10 120 python3 tools/probes/split_dgrad_probe.py bf16 2>&1 | tee "$O/whole.txt"
MRAGAN_DGRAD_SPLIT=1 timeout -k 10 120 python3 tools/probes/split_dgrad_probe.py bf16 2>&1 | tee "$O/split.txt"
MRAGAN_DGRAD_SPLIT=1 timeout -k 10 120 python3 tools/probes/split_dgrad_probe.py fp16 2>&1 | tee "$O/split16.txt"
