#!/bin/bash
# Kernel tests (-k KEXPR) + kbench timing (rocprofv3 kernel trace) + two PMC passes (instruction
# mix, wave-cycle split, LDS) of kbench OPS:   bash tools/gpu_kprof.sh TAG "KEXPR" "OPS" [PREC] [N] [SUBSTR]
set -eo pipefail
TAG=$1; KEXPR=$2; OPS=$3; PREC=${4:-bf16}; KN=${5:-4}; SUB=${6:-mragan}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
bash "$R/tools/gpu_kcheck.sh" "$TAG" "$KEXPR" "$OPS" "$PREC" "$KN"
cd /tmp && export TMPDIR=/tmp
KB="$R/tools/kbench.py --ops $OPS --reps 5 --precision $PREC --N $KN"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d "$O/p1" -o run -- python3 $KB > "$O/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/p2" -o run -- python3 $KB > "$O/p2.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$O" $SUB > "$O/pmc.txt" 2>&1 || true
cat "$O/pmc.txt" | head -40
