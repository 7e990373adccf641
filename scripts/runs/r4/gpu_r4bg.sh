#!/bin/bash
# GPU-box: N4 parity on FIT_G 6, then an isolated A/B of FIT_G 4 / 5 / 6 / 7.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VH_LIB_PATH=$PWD/scratch_libs/fg6.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "n4 or N4 or study or pc or PC or vdp" > gpurun_out/r4bg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4bg_tests.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh fg6 fg4 fg5 fg7 fg6 fg4 fg5 fg7 fg6 fg4 fg5 fg7
