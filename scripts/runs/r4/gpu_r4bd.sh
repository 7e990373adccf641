#!/bin/bash
# GPU-box: fit slice unroll 8 (su8) and the frozen walk's budget 64 / 160 blocks (fr64 / fr160)
# against base (unroll 4, budget 96): isolated A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh base su8 fr64 fr160 base su8 fr64 fr160 base su8 fr64 fr160
