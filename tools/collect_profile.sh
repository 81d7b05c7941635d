#!/bin/bash
# Copy one round's GPU profile (tools/gpu_profile.sh TAG, merged back into gpurun_out/TAG) into
# profiles/ under the TAG prefix: bench line, kernel-trace stats + markdown summary, PMC passes.
#   bash tools/collect_profile.sh r01e
set -euo pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/$TAG
P=$R/profiles
grep '^{' "$O/bench_default.json" > "$P/${TAG}_bench_default.json"
cp "$O/trace/bench_kernel_stats.csv" "$P/${TAG}_bench_kernel_stats.csv"
# the traced bench runs 3 warm-up + 10 timed graph-replayed steps + 2 eager timing steps
python3 "$R/tools/prof_summary.py" --steps 15 --top 40 "$O/trace/bench_kernel_trace.csv" > "$P/${TAG}_bench_kernels.md"
cp "$O/pmc_fetch/run_counter_collection.csv" "$P/${TAG}_res_fwd_pmc_fetch.csv"
cp "$O/pmc_write/run_counter_collection.csv" "$P/${TAG}_res_fwd_pmc_write.csv"
cp "$O/traffic.json" "$P/traffic.json"
echo "profiles/${TAG}_* written"
