#!/bin/bash
# r06u: stride-2 brick variants (weight prefetch 18 steps) — kernel test, then per-variant rocprof kernel
# traces of G down1 / down2 at N = 4 and 2 against the implicit GEMM
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06u
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "stride2_brick" > "$O/kern.log" 2>&1 || { tail -40 "$O/kern.log"; exit 1; }
tail -2 "$O/kern.log"
cd /tmp && export TMPDIR=/tmp
KB="$R/tools/kbench.py --ops down1_fwd16,down1_fwd16s,down2_fwd16,down2_fwd16s --reps 20 --precision bf16"
for N in 4 2; do
  for V in 1 2 4 5; do
    MRAGAN_BRICK_S2_VAR=$V timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_n${N}_v${V}" -o run \
        -- python3 $KB --N $N > "$O/kt_n${N}_v${V}.log" 2>&1
  done
done
echo done
