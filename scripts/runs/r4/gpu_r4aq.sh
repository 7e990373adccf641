#!/bin/bash
# GPU-box: PC pass 0 with the frozen intervals from each block's p range (2 float ops per step):
# N4 parity tests, then an alternated A/B of scratch_libs old / frz / frzs12 (float guess sums).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4aq}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "n4 or N4 or study or pc or PC or vdp" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/dev/ab_libs.sh old frz frzs12 old frz frzs12
