#!/bin/bash
# GPU-box: isolated (one batch in flight) A/B of scratch_libs old / frz / frzs12: per-launch k_n4_study.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh old frz frzs12 old frz frzs12 old frz frzs12
