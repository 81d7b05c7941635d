#!/bin/bash
# Validation pass: kernel A/B vs the baseline library (tools/gpu_lib_ab.sh), then the full -m gpu
# suite and the default bench line without the CPU leg (tools/gpu_iter.sh).
#   bash tools/gpu_val.sh TAG ops
set -eo pipefail
TAG=$1; OPS=$2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_lib_ab.sh "${TAG}_ab" "$OPS"
bash tools/gpu_iter.sh "${TAG}_it" all ""
