#!/bin/bash
# r06af: the stride-2 brick variants re-measured with the 18-step weight prefetch (r06u's run had linked a
# stale 9-step object): rocprof kernel traces of G down1 / down2 at N = 4 and 2 per variant
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06af
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
KB="$R/tools/kbench.py --ops down1_fwd16,down1_fwd16s,down2_fwd16,down2_fwd16s --reps 20 --precision bf16"
for N in 4 2; do
  for V in 1 2 4 5; do
    MRAGAN_BRICK_S2_VAR=$V timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_n${N}_v${V}" -o run \
        -- python3 $KB --N $N > "$O/kt_n${N}_v${V}.log" 2>&1
  done
done
echo done
