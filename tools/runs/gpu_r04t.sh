#!/bin/bash
# r04t: PMC passes on the stride-2 kernels with 16-bit input planes (ABI 14) beside the fp32-input
# forms (bf16, N = 4, 64^3): instruction mix per MFMA and HBM bytes
set -eo pipefail
TAG=${1:-r04t}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
KB="python3 $R/tools/kbench.py --ops down1_fwd,down1_fwd16,down1_wgrad,down1_wgrad16,down2_fwd,down2_fwd16,down2_wgrad,down2_wgrad16 --reps 5 --precision bf16 --N 4"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- $KB > "$O/kt.log" 2>&1
i=0
for c in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$O/p$i" -o run -- $KB > "$O/p$i.log" 2>&1 || echo "pass $i rc $?"
done
python3 $R/tools/pmc_summary.py "$O" igemm wgrad3s2 > "$O/pmc.txt" || true
cat "$O/pmc.txt"
echo "[r04t] done"
