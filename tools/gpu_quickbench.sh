#!/bin/bash
# quick: selected tests + bench (no CPU baseline).  bash tools/gpu_quickbench.sh TAG "pytest -k expr" [bench args]
set -eo pipefail
TAG=$1; KEXPR=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
if [ -n "$KEXPR" ]; then
  step tests 900 python -u -m pytest tests -m gpu -q --tb=short --timeout 300 --timeout-method thread -k "$KEXPR" > "$O/pytest.log" 2>&1
  tail -4 "$O/pytest.log"
fi
step bench 400 python3 bench.py --no-cpu-baseline "$@" > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(d['value'], d['ms_per_step'], d.get('alt_precisions'))
for t in d['top_kernels']:
    print('   ', t)
PY
