#!/bin/bash
# r06n: K-split brick at N = 2 (256 blocks): two-per-CU variant vs one-per-CU (MRAGAN_KS_SMALL_DB1)
# — per-launch kbench, then the same-box step A/B; head data gradient TW 1 / 2 per launch
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/r06n
mkdir -p "$O"
cd "$R"
for N in 2 4; do
  for e in "-" "MRAGAN_KS_SMALL_DB1=1" "MRAGAN_BRICK_KS=2"; do
    envs=""; [ "$e" != "-" ] && envs="$e"
    echo "N=$N $e" >> "$O/kbench.txt"
    env $envs timeout -k 10 120 python3 tools/kbench.py --ops res_fwd16,res_dgrad16s --precision bf16 --N $N --reps 50 \
        >> "$O/kbench.txt" 2>&1
  done
done
for e in "-" "MRAGAN_THIN1_BS_TW1=1"; do
  envs=""; [ "$e" != "-" ] && envs="$e"
  echo "head_dgrad_st N=4 $e" >> "$O/kbench.txt"
  env $envs timeout -k 10 120 python3 tools/kbench.py --ops head_dgrad_st --precision bf16 --N 4 --reps 50 >> "$O/kbench.txt" 2>&1
done
cat "$O/kbench.txt" | grep -v amdgpu.ids
bash tools/gpu_envab.sh r06n/ab 3 "-" "MRAGAN_KS_SMALL_DB1=1"
