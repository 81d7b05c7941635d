#!/bin/bash
# r04p: PMC passes on the stride-2 kernels (bf16, N = 4, 64^3): instruction mix per MFMA and HBM
# bytes (separate --pmc passes, FETCH_SIZE / WRITE_SIZE per the guide's gfx950 correction)
set -eo pipefail
TAG=${1:-r04p}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
KB="python3 $R/tools/kbench.py --ops down1_fwd,down1_wgrad,up2_fwd,down2_fwd,up1_fwd,down2_wgrad --reps 5 --precision bf16 --N 4"
i=0
for c in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
         "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $c --output-format csv -d "$O/p$i" -o run -- $KB > "$O/p$i.log" 2>&1 || echo "pass $i rc $?"
done
python3 $R/tools/pmc_summary.py "$O" igemm brickT wgrad3s2 > "$O/pmc.txt" || true
cat "$O/pmc.txt"
echo "[r04p] done"
