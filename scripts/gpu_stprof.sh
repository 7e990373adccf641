#!/bin/bash
# GPU-box: per-study phase cycles of k_n4_study (scratch_libs/stprof.so: ST_PROF + ST_PROF_ALL, one
# line per study: b, n, iterations, phase cycles) on bench.py's batch.  usage: scripts/gpu_stprof.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-stprof}
VH_LIB_PATH=$PWD/scratch_libs/stprof.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 \
    --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_stprof.json 2> gpurun_out/${TAG}_stprof.err
rc=$?; echo "stprof rc=$rc"; grep -c "ST_PROF b" gpurun_out/${TAG}_stprof.err; exit $rc
