#!/bin/bash
# kbench kernel times of the in-tree library and variant builds (tools/build_variants.sh), same box:
#   bash tools/gpu_var_kb.sh TAG OPS PREC N VARIANT... ("-" = in-tree)
set -eo pipefail
TAG=$1; OPS=$2; PREC=$3; KN=$4; shift 4
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
source "$R/tools/gpu_step.sh"
for v in "$@"; do
  if [ "$v" = "-" ]; then unset MRAGAN_HIP_LIB; else export MRAGAN_HIP_LIB=$R/mra-gan_amd/lib/var/$v/libmragan_hip.so; fi
  step "kb $v" 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_$v" -o run -- python3 "$R/tools/kbench.py" --ops "$OPS" --reps 20 --precision "$PREC" --N "$KN" > "$O/kb_$v.log" 2>&1
  python3 - "$O/kt_$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' in r['Name']:
        print(f"{sys.argv[2]:8s} {float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
done
