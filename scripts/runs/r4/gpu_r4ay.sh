#!/bin/bash
# GPU-box: fit contraction's slice loop unrolled by 4 (su4) and PC pass 0 in 16-step groups (g16)
# against base: N4 parity on su4, then an isolated A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ay}
VH_LIB_PATH=$PWD/scratch_libs/su4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "n4 or N4 or study or pc or PC or vdp" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh base su4 g16 base su4 g16 base su4 g16
