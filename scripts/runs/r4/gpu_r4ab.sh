#!/bin/bash
# GPU-box (round 4): the per-config lines (config 2, config 5, CI, --comm) and their kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash scripts/gpu_lines.sh ${1:-r4ab}
