#!/bin/bash
# GPU-box: k_n4_pcg round counts (scratch_libs/pcgprof.so, -DPCG_PROF) on config 2 and config 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=${1:-pcg}
VH_LIB_PATH=$PWD/scratch_libs/pcgprof.so timeout -k 10 200 python bench.py --shape 256 256 24 --batch 1 --steps 1 --warmup 0 --iso-runs 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_c2.log 2>&1
rc=$?; echo "config2 rc=$rc"; grep -c PCG_PROF gpurun_out/${TAG}_c2.log; [ $rc -eq 0 ] || exit $rc
VH_LIB_PATH=$PWD/scratch_libs/pcgprof.so timeout -k 10 300 python bench.py --shape 512 512 512 --batch 1 --morph3d --steps 1 --warmup 0 --iso-runs 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_c5.log 2>&1
rc=$?; echo "config5 rc=$rc"; grep -c PCG_PROF gpurun_out/${TAG}_c5.log; exit $rc
