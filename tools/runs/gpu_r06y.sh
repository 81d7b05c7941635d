#!/bin/bash
# r06y: res weight gradient with two register sets of staged operands (wgrad3_x3 PF2) — kernel tests, graph
# bit identity, step suites, rocprof kernel traces (PF2 vs MRAGAN_W3_PF1=1), same-box step A/Bs
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06y
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "wgrad" > "$O/kern.log" 2>&1 || { tail -40 "$O/kern.log"; exit 1; }
tail -2 "$O/kern.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py -k "headline or wgrad or overlapped" > "$O/graph.log" 2>&1 || { tail -40 "$O/graph.log"; exit 1; }
tail -2 "$O/graph.log"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_step_gpu.py -k "s64_b2 or s128 or s96" > "$O/steps.log" 2>&1 || { tail -40 "$O/steps.log"; exit 1; }
tail -2 "$O/steps.log"
cd /tmp && export TMPDIR=/tmp
KB="$R/tools/kbench.py --ops res_wgrad16p --reps 20 --precision bf16 --N 4"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_pf2" -o run -- python3 $KB > "$O/kt_pf2.log" 2>&1
MRAGAN_W3_PF1=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_pf1" -o run -- python3 $KB > "$O/kt_pf1.log" 2>&1
grep -h "wgrad3_x3" "$O"/kt_pf2/run_kernel_stats.csv "$O"/kt_pf1/run_kernel_stats.csv | cut -d, -f1-4
cd "$R"
bash tools/gpu_envab.sh r06y/ab 3 "-" "MRAGAN_W3_PF1=1"
BENCH_ARGS="--size 128 --batch 1" bash tools/gpu_envab.sh r06y/ab_128 2 "-" "MRAGAN_W3_PF1=1"
