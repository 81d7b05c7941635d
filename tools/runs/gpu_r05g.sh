#!/bin/bash
# down4 re-check (2 x 8 x 16 bricks) + PMC / stamps of the k7 kernels (stem forward, head dgrad)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/gpu_kcheck.sh" r05g "down4" "dfirst_fwd,stem_fwd,head_dgrad" bf16 4
O=$R/gpurun_out/r05g
cd /tmp && export TMPDIR=/tmp
KB="$R/tools/kbench.py --ops stem_fwd,head_dgrad --reps 5 --precision bf16 --N 4"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d "$O/p1" -o run -- python3 $KB > "$O/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/p2" -o run -- python3 $KB > "$O/p2.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$O" thin1 > "$O/pmc.txt" 2>&1 || true
cat "$O/pmc.txt" | head -40
MRAGAN_STAMPS=1 timeout -k 10 60 python3 "$R/tools/diag_stamps.py" 4 fwd bf16 > "$O/stamps.txt" 2>&1 || true
tail -20 "$O/stamps.txt"
