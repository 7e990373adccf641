#!/bin/bash
# GPU-box quick loop: study-driver parity tests (-k EXPR, default "study"), then a short bench.
# usage: scripts/gpu_quick.sh TAG [pytest -k expr] [extra bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-q}; K=${2:-study}; shift 2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$K" > gpurun_out/quick_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/quick_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/quick_bench_$TAG.json 2> gpurun_out/quick_bench_$TAG.err
rc=$?; echo "bench rc=$rc"; python3 -c "
import json;d=json.loads(open('gpurun_out/quick_bench_$TAG.json').read().strip().splitlines()[-1])
print('VALUE', d['value'], 'ms/step', d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"; exit $rc
