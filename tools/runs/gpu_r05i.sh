#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/gpu_check5.sh" r05i "" "f32" nobench
bash "$R/tools/gpu_kprof.sh" r05i_k "head_dgrad_backward" "stem_fwd_st,head_dgrad_st" bf16 4 thin1r
bash "$R/tools/gpu_envab.sh" r05i_ab 2 "-" "MRAGAN_W3_BLOCKS=128" "MRAGAN_W3_BLOCKS=96" "MRAGAN_W3_BLOCKS=256"
