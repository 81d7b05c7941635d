#!/bin/bash
# r05x: thin1r weight gradient with whole-row P16 loads — k7 tests, kbench (head / stem wgrad,
# res-block kernels for a box-to-box reference against r05k)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r05x
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -rf --tb=short --timeout 120 \
    --timeout-method thread -k "thin1 or k7_planes or stem or head" > "$O/pytest.log" 2>&1
tail -3 "$O/pytest.log"
grep -q " failed" "$O/pytest.log" && exit 1
cd /tmp && export TMPDIR=/tmp
step kt 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/tools/kbench.py" \
    --ops head_wgrad16,stem_wgrad16,res_dgrad16,res_wgrad16,res_fwd16 --reps 10 --precision bf16 --N 4 > "$O/kt.log" 2>&1
python3 - "$O/kt" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'mragan' in r['Name']:
        print(f"{float(r['AverageNs'])/1000:9.2f} us  x{r['Calls']:>4}  {r['Name'][:80]}")
PY
