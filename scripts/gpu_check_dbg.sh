#!/bin/bash
# GPU-box: the -m gpu suite against the DEBUG_BOUNDS library (make DEBUG_BOUNDS=1: every
# data-derived index of the CI kernels checked before its access, the host raising the first
# violation) with a device sync after every launch (VH_SYNC_CHECK=1, naming the launch site of any
# fault).  usage: scripts/gpu_check_dbg.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dbg}
VH_LIB_PATH=vent_analysis_amd/libventhip_dbg.so VH_SYNC_CHECK=1 timeout -k 10 700 \
    python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu_dbg.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest_gpu_dbg.log; exit $rc
