#!/bin/bash
# GPU-box (round 4): ST_PROF phase split after the frozen-mu change, study 3 and block 0 (largest).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ag}
for b in b3 b0; do
  VH_LIB_PATH=$PWD/scratch_ab/stprof_$b.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_$b.json 2> gpurun_out/${TAG}_$b.err
  rc=$?; echo "$b rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep -h ST_PROF gpurun_out/${TAG}_$b.json
done
