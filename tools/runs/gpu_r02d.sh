#!/bin/bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02d
mkdir -p "$O"
cd "$R"
echo "[r02d] kernels + boundary tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --tb=short --timeout 300 --timeout-method thread -k "kernels or checkpoint or dp_two or graph_step or sliding" > "$O/pytest.log" 2>&1 || { tail -80 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
echo "[r02d] precision envelopes"
timeout -k 10 600 python -u tools/precision_envelope.py step_r9_s32_b1 step_r6_s24_b2_nc2_lsgan step_r9_s32_b2_ngf16 step_unet_s32_b2_ngf8 step_r9_s64_b2 --out "$O/envelope.json" 2>&1 | grep '^{' 
