#!/bin/bash
# GPU-box: rows per group in the fit / eval walks (FIT_G 6 / 8 / 12): isolated A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh base fg6 fg12 base fg6 fg12 base fg6 fg12
