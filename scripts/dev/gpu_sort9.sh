#!/bin/bash
# GPU-box: scratch_libs/s9.so (9-bit-digit sort skipping constant digit positions): the whole GPU
# suite on it, the VS_PROF split (scratch_libs/vsprof.so, same source), then the headline A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VH_LIB_PATH=scratch_libs/s9.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests > gpurun_out/r6n_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6n_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/dev/gpu_vsprof.sh || exit 1
bash scripts/gpu_ab_headline.sh r6nh s9
