#!/bin/bash
# r04h: instruction-fetch counters on the K-split brick (is the straight-line prologue / epilogue
# bound by instruction-cache misses?) + the full default bench line (legs incl. 96^3 nc2 fp16 and
# unet_custom 64^3)
set -eo pipefail
TAG=${1:-r04h}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
step list 60 rocprofv3 -L > "$O/counters.txt" 2>&1
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_INST[A-Z_]*" "$O/counters.txt" | sort -u > "$O/counters_ifetch.txt" || true
cat "$O/counters_ifetch.txt" | tr '\n' ' '; echo
KB="python3 $R/tools/kbench.py --ops res_fwd16,res_dgrad16 --reps 5 --precision bf16 --N 4"
for c in "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA"; do
  n=$(echo $c | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$n" -o run -- $KB > "$O/pmc_$n.log" 2>&1) || echo "pmc $n failed"
done
python3 tools/pmc_summary.py "$O" brick > "$O/pmc.txt" || true; cat "$O/pmc.txt"
step bench 900 python3 bench.py > "$O/bench.json" 2> "$O/bench.err"
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("head", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["step_roofline"])
for k, v in d.get("legs", {}).items():
    print("leg", k, v["value"], v["ms_per_step"], v.get("roofline", {}).get("frac"))
print("alt", {k: v["ms_per_step"] for k, v in d.get("alt_precisions", {}).items()})
print("cpu", d.get("cpu_baseline", {}).get("value"))
PY
echo "[r04h] done"
