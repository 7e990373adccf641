#!/bin/bash
# GPU-box: probe of pass 0's double exp cost (fexp: __expf, not the spec's floats) vs base, isolated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh base fexp base fexp base fexp
