#!/bin/bash
# GPU-box (round 4): same-box A/B of the eval row-weight batching (r4aa's box ran slower overall):
# base, evb, base, evb -- one-batch and two-in-flight bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ae}
for v in base evb base evb; do
  VH_LIB_PATH=$PWD/scratch_ab/$v.so timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_tmp.json 2> /dev/null
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/${TAG}_tmp.json') if l.startswith('{')][-1]); print('$v', d['value'], d['n4_study_times']['mean_us'], d['roofline']['isolated']['avg_launch_us'])" | tee -a gpurun_out/${TAG}_ab.txt
done
