#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/gpu_kprof.sh" r05h "thin1 or k7 or head_dgrad or stem" "stem_fwd_st,head_dgrad_st" bf16 4 thin1r
bash "$R/tools/gpu_envab.sh" r05h_ab 2 "-" "MRAGAN_W3_BLOCKS=128" "MRAGAN_W3_BLOCKS=96" "MRAGAN_W3_BLOCKS=256"
