#!/bin/bash
# GPU-box: the one-study lines (config 2 shape and one 128x128x24 study) for MODES at INFL batches in flight.
# usage: [MODES="sweep grid"] [INFL="1 3"] scripts/gpu_grid_check_lines.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
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
