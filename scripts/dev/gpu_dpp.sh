#!/bin/bash
# GPU-box: grid-PC DPP wave-scan variant (scratch_libs/pcgdpp.so): parity tests, then config 2 / config 5 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VH_LIB_PATH=scratch_libs/pcgdpp.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py -k "n4 or grid or config2 or pcg or sort or vdp or bench" > gpurun_out/r6d_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6d_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_config2.sh r6d2 pcgdpp && bash scripts/gpu_ab_c5.sh r6d5 pcgdpp && \
bash scripts/gpu_ab_headline.sh r6dh pcgdpp
