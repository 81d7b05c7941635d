#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/gpu_check5.sh" r05l "instnorm or in_launch or op16_instnorm" "" nobench
bash "$R/tools/gpu_envab.sh" r05l_ab 3 "-" "MRAGAN_IN_APPLY3=0"
