#!/bin/bash
# out-of-bounds write probe of the ResnetBlock data gradient: whole-grid brick and split
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bo}
mkdir -p "$O"
cd "$R"
timeout -k 10 120 python3 tools/probes/oob_probe.py bf16 2>&1 | tee "$O/whole.txt" || true
MRAGAN_DGRAD_SPLIT=1 timeout -k 10 120 python3 tools/probes/oob_probe.py bf16 2>&1 | tee "$O/split.txt" || true
