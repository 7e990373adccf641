#!/bin/bash
# GPU-box: study-driver parity tests, then bench in both N4 modes and a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "study" > gpurun_out/study_tests.log 2>&1
rc=$?; echo "study tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --n4-mode study > gpurun_out/bench_study.json 2> gpurun_out/bench_study.err
rc=$?; echo "bench study rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_study -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --n4-mode study > gpurun_out/prof_study.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
