#!/bin/bash
# GPU-box: stage 0's round cap before the frozen walk (PC_AMAX0 28 / 40 / 56) with the drift-seeded
# guesses: isolated A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh base am28 am56 base am28 am56 base am28 am56
