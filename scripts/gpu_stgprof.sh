#!/bin/bash
# GPU-box: phase split of the grid study form (STG_PROF builds in scratch_libs/), one-study runs.
# usage: scripts/gpu_stgprof.sh TAG LIB [SHAPES]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; LIB=$2
for shape in ${SHAPES:-"256 256 24" "128 128 24"}; do :; done
for s in 256x256x24 128x128x24; do
  sh=${s//x/ }
  VH_LIB_PATH=scratch_libs/$LIB.so timeout -k 10 200 python3 bench.py --shape $sh --batch 1 --steps 2 --warmup 1 \
      --inflight 1 --iso-runs 1 --no-cpu-baseline --no-h2h --n4-mode grid > gpurun_out/${TAG}_${LIB}_$s.log 2>&1
  rc=$?; echo "$s rc=$rc"; grep -c STG_PROF gpurun_out/${TAG}_${LIB}_$s.log; [ $rc -eq 0 ] || exit $rc
done
