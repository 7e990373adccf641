#!/bin/bash
# GPU-box (round 4): batches in flight on the final build, 2 vs 3, alternated on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ai}
for v in 2 3 2 3; do
  timeout -k 10 300 python bench.py --steps 12 --warmup 3 --inflight $v --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_tmp.json 2> /dev/null
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/${TAG}_tmp.json') if l.startswith('{')][-1]); print('inflight $v', d['value'], d['ms_per_step'], d['batch_latency_ms'])" | tee -a gpurun_out/${TAG}_ab.txt
done
