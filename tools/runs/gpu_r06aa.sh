#!/bin/bash
# r06aa: re-check of launch-plan A/B switches on the round-6 four-stream step (bf16 64³ b2), same box,
# alternating: the res weight-gradient block budget, the one-per-CU K-split variant for small grids, the
# implicit-GEMM minimum block count
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/gpu_envab.sh r06aa/ab 2 "-" "MRAGAN_W3_BLOCKS=256" "MRAGAN_W3_BLOCKS=128" "MRAGAN_KS_SMALL_DB1=1" \
    "MRAGAN_IG_MINBLOCKS=256" "MRAGAN_IG_MINBLOCKS=1024"
