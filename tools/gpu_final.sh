#!/bin/bash
# Evidence at HEAD: all -m gpu tests, smoke, the default (driver) bench line (full report to a file),
# a kernel trace of the headline workload (traced durations include the other lane's contention),
# and PMC passes (FETCH_SIZE / WRITE_SIZE; instruction mix) of the res-block operand-plane kernels
# (bf16, N = 4).
#   bash tools/gpu_final.sh TAG [notests]
set -eo pipefail
TAG=${1:-r04final}
NOTESTS=${2:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
if [ -z "$NOTESTS" ]; then
  step tests 900 python3 -u -m pytest tests -m gpu -q -rf --tb=short --timeout 300 --timeout-method thread \
      > "$O/pytest.log" 2>&1
  tail -3 "$O/pytest.log"
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  tail -2 "$O/smoke.log"
fi
step bench 700 python3 bench.py --full-out "gpurun_out/$TAG/bench_full.json" > "$O/bench.json" 2> "$O/bench.err"
cut -c1-400 "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o bench \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-kernel-timing --alt-precisions '' --legs '' --no-cpu-baseline \
    > "$O/trace.log" 2>&1
KB="$R/tools/kbench.py --ops res_wgrad16p,res_dgrad16s,res_fwd16,down1_fwd16,down2_fwd16s,down1_wgrad16 --reps 10 --precision bf16 --N 4"
step ktrace 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace" -o run -- python3 $KB > "$O/ktrace.log" 2>&1
step fetch 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o run -- python3 $KB > "$O/fetch.log" 2>&1
step write 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o run -- python3 $KB > "$O/write.log" 2>&1
step mix 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY --output-format csv -d "$O/mix" -o run -- python3 $KB > "$O/mix.log" 2>&1
# LDS pass (the res weight gradient's staging stores + transposing reads): array cycles and conflicts
step lds 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES \
    --output-format csv -d "$O/lds" -o run -- python3 $KB > "$O/lds.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$O" brick wgrad igemm > "$O/pmc.txt" || true
echo "[final] done"
