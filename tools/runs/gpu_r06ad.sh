#!/bin/bash
# r06ad: launch-class timing by graph replay — the default bench line (classes graph-timed) and the same
# run with MRAGAN_EAGER_CLASS_TIMING=1, same box; the torch.ops / kernel-timer tests
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06ad
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 bench.py --legs '' --alt-precisions '' --no-cpu-baseline --full-out "$O/full_graph.json" > "$O/graph.json" 2> "$O/graph.err" || { tail -30 "$O/graph.err"; exit 1; }
MRAGAN_EAGER_CLASS_TIMING=1 timeout -k 10 600 python3 bench.py --legs '' --alt-precisions '' --no-cpu-baseline --full-out "$O/full_eager.json" > "$O/eager.json" 2> "$O/eager.err" || { tail -30 "$O/eager.err"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for t in ("graph", "eager"):
    d = json.load(open(f"{O}/{t}.json"))
    print(t, d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel"][-40:], d["kernel_ms_per_step_serial"])
    for k in d["top_kernels"][:6]:
        print("   ", k)
PY
