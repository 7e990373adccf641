#!/bin/bash
# GPU-box: ONE rocprofv3 --pmc pass of one config's workload, as the call's last GPU step: with the
# cooperative grid-PC launch (configs 2 and 5) rocprofv3 segfaults at exit after writing the
# counters (rc 139), after which nothing more may run on the GPU in that call.  A 139 with the
# counter CSV present counts as the pass done.  The FETCH_SIZE and WRITE_SIZE directories of two
# calls are then summarised on the CPU: BENCH_ARGS="<workload>" python scripts/pmc_summary.py OUT DIR1 DIR2
# usage: scripts/gpu_pmc1.sh TAG COUNTER "BENCH ARGS"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; C=$2; ARGS=$3
timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex 'k_n4_|k_plane|k_sort|k_kmeans' --output-format csv \
    -d gpurun_out/${TAG}_$C -o pmc -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --iso-runs 1 \
    --no-cpu-baseline --no-profile --no-h2h $ARGS > gpurun_out/${TAG}_$C.log 2>&1
rc=$?; echo "pmc $C rc=$rc"
if [ $rc -eq 139 ] && [ -s gpurun_out/${TAG}_$C/pmc_counter_collection.csv ]; then
  echo "rocprofv3's exit-time segfault after the counters were written (cooperative launch)"; exit 0
fi
exit $rc
