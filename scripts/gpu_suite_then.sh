#!/bin/bash
# GPU-box: the -m gpu suite (one process), then the given scripts in order.  Test failures (pytest
# rc 1) do not stop the later steps; any other non-zero status (a fault, abort, timeout) does.
# usage: scripts/gpu_suite_then.sh TAG "script1 args" "script2 args" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for step in "$@"; do
  bash $step
  rc=$?; echo "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
