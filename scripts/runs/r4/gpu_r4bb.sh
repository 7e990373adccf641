#!/bin/bash
# GPU-box: stage 0's round cap PC_AMAX0 20 / 24 / 28: isolated A/B; N4 parity on am20.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VH_LIB_PATH=$PWD/scratch_libs/am20.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "n4 or N4 or study or pc or PC or vdp" > gpurun_out/r4bb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4bb_tests.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh am28 am20 am24 am28 am20 am24 am28 am20 am24
