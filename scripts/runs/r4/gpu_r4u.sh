#!/bin/bash
# GPU-box (round 4): per-study PC rounds and serial fallbacks against per-study time (one batch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4u}
VH_STUDY_TRACE=gpurun_out/${TAG}_trace.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/study_pc.py gpurun_out/${TAG}_trace.csv
