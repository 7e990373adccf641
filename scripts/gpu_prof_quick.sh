#!/bin/bash
# GPU-box: rocprofv3 kernel trace + stats of a short default bench (no CPU baseline / host-to-host);
# extra arguments go to bench.py.  usage: scripts/gpu_prof_quick.sh TAG [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2h "$@" > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$TAG.err; exit $rc; }
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/${TAG}_kernel_stats.csv
python3 -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:24]: print('%-60s %6s %12.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))" gpurun_out/${TAG}_kernel_stats.csv
