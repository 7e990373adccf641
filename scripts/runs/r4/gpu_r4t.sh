#!/bin/bash
# GPU-box (round 4): PC_PROF of the default build (block 0 = the largest study: pass 0, stage-0
# rounds, PCX, phase B per iteration) and ST_PROF of study 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4t}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
VH_LIB_PATH=$PWD/scratch_libs/pcprof.so run pcprof python bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-h2h
VH_LIB_PATH=$PWD/scratch_libs/stprof_b3.so run stprof python bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-h2h
grep -c PCW_PROF gpurun_out/${TAG}_pcprof.json
grep -h "ST_PROF" gpurun_out/${TAG}_stprof.json
