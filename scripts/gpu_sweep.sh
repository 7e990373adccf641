#!/bin/bash
# GPU-box: parity tests then a sub-batch sweep of the bench (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for sb in ${SWEEP:-0 128 64}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --subbatch $sb > gpurun_out/sweep_$sb.json 2> gpurun_out/sweep_$sb.err
  rc=$?; echo "sweep $sb rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
