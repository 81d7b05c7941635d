#!/bin/bash
# r06l: hardware queues per process (HIP runtime's GPU_MAX_HW_QUEUES, 4 by default on the box)
# against the replayed 4-branch step graph: same-box A/B (result: profiles/r06/r06l_hw_queues.txt;
# the =2 arm segfaulted at start-up, so the run ended after arm 2)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd "$R"
bash tools/gpu_envab.sh r06l/ab 2 "-" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=2"
