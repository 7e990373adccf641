#!/bin/bash
# GPU-box (round 4): PC pass 0 with 16-step transpose groups (PC_G0=16, half the barriers) against
# 8 -- parity of the variant, then base / g16 / base / g16 bench lines on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ah}
VH_LIB_PATH=$PWD/scratch_ab/g16.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "study or bench_workload or n4 or pc or sweep" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "g16 tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base g16 base g16; do
  VH_LIB_PATH=$PWD/scratch_ab/$v.so timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_tmp.json 2> /dev/null
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; exit $rc; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/${TAG}_tmp.json') if l.startswith('{')][-1]); print('$v', d['value'], d['n4_study_times']['mean_us'], d['n4_study_times']['max_us'], d['roofline']['isolated']['avg_launch_us'])" | tee -a gpurun_out/${TAG}_ab.txt
done
