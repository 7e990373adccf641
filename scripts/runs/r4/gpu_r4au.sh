#!/bin/bash
# GPU-box: PC_PROF rounds of the largest study and the ST_PROF phase split of study 118 with the
# drift-seeded guesses.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
bash scripts/dev/pc_prof.sh || exit 1
VARIANTS="stprof118" BENCH_ARGS="--inflight 1" bash scripts/dev/phase_ab.sh
