#!/bin/bash
# Same-box kernel A/B of an environment switch on kbench ops (kernel trace each):
#   bash tools/gpu_env_ab.sh TAG VAR=VALUE op1,op2   (KB_ARGS: extra kbench arguments)
set -eo pipefail
TAG=$1; SETTING=$2; OPS=$3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
for side in off on; do
  if [ $side = on ]; then export "$SETTING"; fi
  step "kbench $side" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$side" -o run -- python3 tools/kbench.py --ops "$OPS" --reps 20 --precision bf16x3 ${KB_ARGS:-} > "$O/kbench_$side.log" 2>&1
  python3 - "$O/kt_$side" "$side" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r['Name'].startswith('void at::') or 'rocclr' in r['Name']:
        continue
    print(f"{sys.argv[2]:4s} {float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
done
