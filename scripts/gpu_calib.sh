#!/bin/bash
# GPU-box: FETCH_SIZE / WRITE_SIZE calibration per access form (scripts/microbench/fetch_calib.hip,
# VERDICT r5 item 3).  One rocprofv3 --pmc pass per (mode, counter), then scripts/calib_summary.py.
# usage: scripts/gpu_calib.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
for m in 0 1 2 3 4 5 6; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_calib_m${m}_$c -o pmc -- \
        ./scripts/microbench/fetch_calib $m > gpurun_out/${TAG}_calib_m${m}_$c.log 2>&1
    rc=$?; echo "mode $m $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 scripts/calib_summary.py gpurun_out/${TAG}_calib gpurun_out/${TAG}_fetch_calib.json
