#!/bin/bash
# GPU-box (round 4): the CI line under rocprofv3 kernel + memory-copy traces (where 0.22 ms go).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4al}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --workload ci --steps 20 --warmup 3 > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
ls gpurun_out/${TAG}_prof
