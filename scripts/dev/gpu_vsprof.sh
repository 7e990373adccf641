#!/bin/bash
# GPU-box: the VS_PROF phase split of k_sort_vol (scratch_libs/vsprof.so), one bench step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
VH_LIB_PATH=$PWD/scratch_libs/vsprof.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --iso-runs 1 --no-cpu-baseline --no-h2h \
    > gpurun_out/vsprof.out 2> gpurun_out/vsprof.err
rc=$?; [ $rc -eq 0 ] || exit $rc
grep VSPROF gpurun_out/vsprof.out | head -4
