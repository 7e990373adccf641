#!/bin/bash
# GPU-box: scratch_libs/fitq.so (fit row offsets before the group's loads): N4 parity subset, then the
# headline and config-5 A/B against the tree's library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VH_LIB_PATH=scratch_libs/fitq.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py -k "n4 or config2 or bench" > gpurun_out/r6f_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6f_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_headline.sh r6fh fitq && bash scripts/gpu_ab_c5.sh r6f5 fitq
