#!/bin/bash
# GPU-box: sort parity subset with scratch_libs/$VAR.so, the VS_PROF phase split, then an alternated
# --no-n4 A/B of base vs $VAR.  usage: VAR=vsr3 scripts/dev/gpu_sort.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
VH_LIB_PATH=$PWD/scratch_libs/$VAR.so timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "sort or adversarial or kmeans or class or vdp or mean" > gpurun_out/sort_pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sort_pytest.log; [ $rc -eq 0 ] || exit $rc
VH_LIB_PATH=$PWD/scratch_libs/vsprof.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --iso-runs 1 --no-cpu-baseline --no-h2h \
    > gpurun_out/vsprof.out 2> gpurun_out/vsprof.err
rc=$?; [ $rc -eq 0 ] || exit $rc
grep VSPROF gpurun_out/vsprof.out | head -4
VARIANTS="base $VAR" REPS=2 BENCH_ARGS="--no-n4" bash scripts/gpu_ab.sh sort
