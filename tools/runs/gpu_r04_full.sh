#!/bin/bash
# Round-4 HEAD check: the whole GPU suite (the driver's round-end tier) and smoke()
set -eo pipefail
TAG=${1:-r04_full}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step tests 1000 python3 -u -m pytest tests -m gpu -q -rfs --tb=short --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
tail -8 "$O/pytest.log"
step smoke 150 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
tail -3 "$O/smoke.log"
echo "[r04_full] done"
