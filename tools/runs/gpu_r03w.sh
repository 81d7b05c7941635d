#!/bin/bash
# r03w: PMC probe of the ResnetBlock classes at HEAD (bf16, N=4)
set -eo pipefail
TAG=${1:-r03w}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
PREC=bf16 KN=4 bash tools/pmc_probe.sh "$TAG/pmc" res_fwd16,res_dgrad16,res_wgrad16
echo "[r03w] done"
