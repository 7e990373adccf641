#!/bin/bash
# GPU-box: scratch_libs/mstat.so (grid-PC DPP scan + LDS peer match in the sort + mask stats rework):
# the whole GPU suite on it, then the headline A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VH_LIB_PATH=scratch_libs/mstat.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    -m gpu tests > gpurun_out/r6m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6m_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_headline.sh r6mh mstat
