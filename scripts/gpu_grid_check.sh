#!/bin/bash
# GPU-box: the grid form's parity tests first (fast failure), then the whole -m gpu suite, then the
# one-study lines (config 2 shape and one 128x128x24 study) for the sweep driver and the grid form at
# 1 and 3 batches in flight.  Stops at the first failure.
# usage: scripts/gpu_grid_check.sh TAG [SKIP_SUITE=1]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k grid > gpurun_out/${TAG}_grid_tests.log 2>&1
rc=$?; echo "grid tests rc=$rc"; tail -2 gpurun_out/${TAG}_grid_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for shape in "256 256 24" "128 128 24"; do
  for m in ${MODES-sweep grid}; do
    for inf in ${INFL-1 3}; do
      s=${shape// /x}
      timeout -k 10 300 python3 bench.py --shape $shape --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-h2h \
          --n4-mode $m --inflight $inf > gpurun_out/${TAG}_${s}_${m}_i$inf.json 2> gpurun_out/${TAG}_${s}_${m}_i$inf.err
      rc=$?; [ $rc -eq 0 ] || { echo "bench $s $m $inf rc=$rc"; tail -3 gpurun_out/${TAG}_${s}_${m}_i$inf.err; exit $rc; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline'] or {}; print(sys.argv[2], d['value'], 'vol/s', d['ms_per_step'], 'ms/step lat', d['batch_latency_ms'], r.get('kernel'), r.get('avg_launch_us'), r.get('frac'))" gpurun_out/${TAG}_${s}_${m}_i$inf.json "$s $m inflight $inf"
    done
  done
done
