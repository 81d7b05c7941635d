set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc1
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/p1 -o run -- python3 $R/tools/kbench.py --ops res_fwd,res_dgrad,res_wgrad --reps 5 --precision bf16x3 > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $R/tools/kbench.py --ops res_fwd,res_dgrad,res_wgrad --reps 5 --precision bf16x3 > $O/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/tools/kbench.py --reps 10 --precision bf16x3 > $O/t.log 2>&1
