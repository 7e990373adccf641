#!/bin/bash
# GPU-box: the 512-thread study build (scratch_libs/t512.so: two studies per CU) against the tree's
# 1024-thread library at the default bench, then the variant at 4 and 6 batches in flight
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VH_LIB_PATH=scratch_libs/t512.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py -k "n4 and not grid" > gpurun_out/r6t_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6t_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_headline.sh r6th t512 || exit 1
for inf in 4 6; do
  VH_LIB_PATH=scratch_libs/t512.so timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h \
      --inflight $inf > gpurun_out/r6t_inf$inf.json 2> gpurun_out/r6t_inf$inf.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('t512 inflight', sys.argv[2], d['value'], d['ms_per_step'], d['n4_study_times'])" gpurun_out/r6t_inf$inf.json $inf
done
