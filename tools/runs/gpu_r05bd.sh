#!/bin/bash
# instruction-cache counters of the res-block kernels (kbench, bf16, 64³ b2 shapes N = 2 and 4):
# is the K-split brick's first pass over its 27 KB unrolled body fetch-bound?
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/${1:-r05bd}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for N in 2 4; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH \
    --output-format csv -d "$O/n$N" -o run -- python3 "$R/tools/kbench.py" --ops res_fwd16,res_dgrad16 --reps 5 --precision bf16 --N $N > "$O/n$N.log" 2>&1 || { echo "pmc rc $?"; tail -5 "$O/n$N.log"; exit 1; }
  python3 "$R/tools/pmc_summary.py" "$O/n$N" mragan > "$O/n$N.txt" 2>&1 || true
  cat "$O/n$N.txt"
done
