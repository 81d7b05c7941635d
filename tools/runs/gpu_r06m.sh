#!/bin/bash
# r06m: head data gradient (thin1r EPI 2) at two blocks per CU with its backward statistics in the
# store layout — kernel + step tests, then same-box A/B against one block per CU
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06m
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "head_dgrad or thin1 or in_stats_partials or stats" > "$O/kern.log" 2>&1
tail -2 "$O/kern.log"
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_graph_gpu.py tests/test_step_gpu.py > "$O/steps.log" 2>&1
tail -2 "$O/steps.log"
bash tools/gpu_envab.sh r06m/ab 3 "-" "MRAGAN_THIN1_BS_TW1=1"
# K-split brick phase stamps at the bench shapes (N = 4 / 2), for the N = 2 res forward / dgrad
timeout -k 10 120 python3 tools/diag_ks.py bf16 > "$O/diag_ks.txt" 2>&1
cat "$O/diag_ks.txt"
# HBM traffic of the paired res weight gradient (the dominant class since round 6): two PMC passes
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
    -- python3 "$R/tools/kbench.py" --ops res_wgrad16p --precision bf16 --reps 10 > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run \
    -- python3 "$R/tools/kbench.py" --ops res_wgrad16p --precision bf16 --reps 10 > "$O/pmc_write.log" 2>&1
cd "$R"
python3 tools/pmc_traffic.py --fetch "$O/pmc_fetch" --write "$O/pmc_write" --kernel "wgrad3_x3_kernel<128;wgrad_reduce" \
    --key "wgrad3_x3(op16);wgrad_reduce|wgrad 128x128 k3 s1 [4+2x16x16x16]" --algorithmic-bytes 17018880 \
    --source "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tools/kbench.py --ops res_wgrad16p --precision bf16 (N=4+2; reduce launches paired with their producer), profiles/r06" \
    --out "$O/traffic.json"
