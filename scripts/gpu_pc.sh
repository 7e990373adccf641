#!/bin/bash
# GPU-box check of the PC convergence chain: exhaustive step-constant check, N4 parity tests
# (-k EXPR), then a short bench.  usage: scripts/gpu_pc.sh TAG [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pc}; K=${2:-n4}
timeout -k 10 60 ./scripts/microbench/recip_exact > gpurun_out/${TAG}_recip.log 2>&1
rc=$?; cat gpurun_out/${TAG}_recip.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$K" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench.json; exit $rc
