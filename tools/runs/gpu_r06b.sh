#!/bin/bash
# r06b: one ResnetBlock weight gradient per conv per generator (first + cycle pass, ABI 19 pair):
# kernel tests, graph-vs-eager tests, the step suites (all but the 64³ b2 case, whose precision
# fixture is being regenerated), headline bench + a same-box A/B with the pairing off
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06b
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step kern 300 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 --timeout-method thread \
    -k "wgrad or interior_shell or null_fp32 or stale_fp32" > "$O/kern.log" 2>&1
tail -3 "$O/kern.log"
step graph 600 python3 -u -m pytest tests/test_graph_gpu.py tests/test_dp_gpu.py -m gpu -q -rf --tb=short -s --timeout 300 \
    --timeout-method thread > "$O/graph.log" 2>&1
tail -3 "$O/graph.log"
step steps 900 python3 -u -m pytest tests/test_step_gpu.py -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread \
    -k "not s64_b2" > "$O/steps.log" 2>&1
tail -3 "$O/steps.log"
bash tools/gpu_envab.sh r06b/ab 2 "-" "MRAGAN_NO_WGRAD_DEFER=1"
step bench 300 python3 bench.py --steps 30 --warmup 5 --alt-precisions '' --no-cpu-baseline --full-out "gpurun_out/r06b/bench_full.json" \
    > "$O/bench.json" 2> "$O/bench.err"
cut -c1-300 "$O/bench.json"
