#!/bin/bash
# r05p: thin1r forward with register weights / fragment prefetch / stores after the statistics —
# thin1 kernel tests + kbench timing and PMC of the stem forward and head data gradient
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/gpu_kprof.sh" r05p "thin1 or head_dgrad or k7_planes or stem" "stem_fwd_st,head_dgrad_st,head_wgrad16,stem_wgrad16" bf16 4 thin1r
