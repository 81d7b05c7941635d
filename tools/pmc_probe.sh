#!/bin/bash
# PMC probe of selected kbench ops (GPU box): stall / MFMA / LDS counters and HBM traffic.
#   bash tools/pmc_probe.sh TAG OPS
set -euo pipefail
TAG=${1:-pmc}
OPS=${2:-res_fwd}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
KB="python3 $R/tools/kbench.py --ops $OPS --reps 5 --precision ${PREC:-bf16x3} --N ${KN:-4}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d "$O/p1" -o run -- $KB > "$O/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d "$O/p2" -o run -- $KB > "$O/p2.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/p3" -o run -- $KB > "$O/p3.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/p4" -o run -- $KB > "$O/p4.log" 2>&1
echo "[pmc_probe] done"
