#!/bin/bash
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02e
mkdir -p "$O"
cd "$R"
source tools/gpu_step.sh
step envelope 600 python -u tools/precision_envelope.py step_r9_s32_b1 step_r6_s24_b2_nc2_lsgan step_r9_s32_b2_ngf16 step_unet_s32_b2_ngf8 step_r9_s64_b2 --out "$O/envelope.json"
step tests 600 python -u -m pytest tests -m gpu -q --tb=short --timeout 300 --timeout-method thread -k "checkpoint or dp_two or thin or test_conv3d_fwd or test_conv3d_dgrad" -o log_cli=false
