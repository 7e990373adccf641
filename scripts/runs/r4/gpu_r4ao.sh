#!/bin/bash
# GPU-box (round 4): CI map and scalars stored by the kernels into device-mapped page-locked host memory -- CI / class / pickle
# tests, then the CI line twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ao}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ci or CI or class or pickle" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload ci --steps 40 --warmup 5 > gpurun_out/${TAG}_ci$i.json 2> gpurun_out/${TAG}_ci$i.err
  rc=$?; echo "ci$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/${TAG}_ci$i.json') if l.startswith('{')][-1]); print('ci$i', d['ms_per_step'], {k: (v['seconds_per_map'], v['ci_walk_us']) for k, v in d['config']['cases'].items()})"
done
