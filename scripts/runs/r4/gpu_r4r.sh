#!/bin/bash
# GPU-box (round 4 evidence): rocprofv3 kernel-trace statistics of the default bench (no PMC), then
# the FETCH_SIZE / WRITE_SIZE passes (each its own run) for roofline.traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4r}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh ${TAG}_pmc
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cat gpurun_out/${TAG}_pmc_summary.log
find gpurun_out/${TAG}_trace -name "*kernel_stats.csv" | head -3
