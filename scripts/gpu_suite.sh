#!/bin/bash
# GPU-box: the -m gpu suite (one process), then a short bench line.  usage: scripts/gpu_suite.sh TAG [BENCH_ARGS...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-suite}; shift
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; cat gpurun_out/${TAG}_bench.json; exit $rc
