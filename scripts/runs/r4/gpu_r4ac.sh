#!/bin/bash
# GPU-box (round 4): CI host-to-host after the fused clears, the parallel percentile and the output
# pinned in place (A/B: VH_CI_STAGE=1), with the CI parity tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ac}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ci or CI" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for v in pin stage pin2; do
  if [ $v = stage ]; then export VH_CI_STAGE=1; else unset VH_CI_STAGE; fi
  timeout -k 10 300 python bench.py --workload ci --steps 40 --warmup 5 > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/${TAG}_$v.json') if l.startswith('{')][-1]); print('$v', d['ms_per_step'], {k: (v['seconds_per_map'], v['ci_walk_us']) for k, v in d['config']['cases'].items()})"
done
