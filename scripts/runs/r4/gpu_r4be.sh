#!/bin/bash
# GPU-box: batches in flight 3 vs 4 on the final build, alternated three times (device-resident line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for k in 3 4; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-h2h --inflight $k > gpurun_out/r4be_if${k}_$r.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/r4be_if${k}_$r.json').read().strip().splitlines()[-1]);print('inflight $k', d['value'], d['ms_per_step'])"
  done
done
