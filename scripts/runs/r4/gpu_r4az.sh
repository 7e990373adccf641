#!/bin/bash
# GPU-box: E map variants against base -- wpre (Wiener gains by the whole workgroup) and gexp (the
# Gaussian kernel's exp by vh_expf_any): N4 parity on each, then an isolated A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4az}
for v in wpre gexp; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "n4 or N4 or study or pc or PC or vdp" > gpurun_out/${TAG}_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -1 gpurun_out/${TAG}_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
AB_ARGS="--inflight 1 --steps 10" bash scripts/dev/ab_libs.sh base wpre gexp base wpre gexp base wpre gexp
