#!/bin/bash
# Same-box kernel A/B by environment switch: kbench ops under a rocprofv3 kernel trace, once per
# "VAR=VALUE[;VAR=VALUE]" setting ("-" = none), printing each kernel's mean.
#   bash tools/gpu_ab_env.sh TAG PREC N OPS "- MRAGAN_X=1"
set -eo pipefail
TAG=$1; PREC=$2; N=$3; OPS=$4; SETS=${5:-"-"}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
source tools/gpu_step.sh
i=0
for e in $SETS; do
  i=$((i + 1))
  envs=()
  if [ "$e" != "-" ]; then IFS=';' read -ra envs <<< "$e"; envs=(env "${envs[@]}"); fi
  step "kb $e" 120 "${envs[@]}" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$i" -o run -- \
      python3 tools/kbench.py --ops "$OPS" --reps 20 --precision "$PREC" --N "$N" > "$O/kb_$i.log" 2>&1
  python3 - "$O/kt_$i" "$e" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' in r['Name']:
        print(f"{sys.argv[2]:>24s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
done
echo "[ab] done"
