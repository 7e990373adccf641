#!/bin/bash
# GPU-box: round-6 closing lines besides the default bench (which gpu_evidence.sh makes): config 2
# (grid form), config 5, one 128x128x24 study per batch, the class call latency, CI, the one-rank
# RCCL path; then ONE rocprofv3 kernel trace (TRACE=config2|config5, --inflight 1), last in the call
# (rocprofv3's exit-time fault after cooperative launches).
# usage: [TRACE=config2] scripts/gpu_final_lines.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
declare -A A
A[config2]="--shape 256 256 24 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-h2h"
A[config5]="--shape 512 512 512 --batch 1 --morph3d --steps 3 --warmup 1 --no-cpu-baseline --no-h2h"
A[one]="--shape 128 128 24 --batch 1 --steps 20 --warmup 3 --no-cpu-baseline --no-h2h"
A[class]="--workload class --steps 20 --warmup 3"
A[ci]="--workload ci --steps 20 --warmup 3"
A[comm1]="--comm --steps 5 --warmup 1 --no-cpu-baseline --no-h2h"
for name in ${LINES-config2 config5 one class ci comm1}; do
  timeout -k 10 600 python3 bench.py ${A[$name]} > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${name}.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], r.get('kernel'), r.get('frac'), r.get('traffic_over_alg'))" gpurun_out/${TAG}_${name}.json $name
done
if [ -n "${TRACE-}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${TRACE}_prof -o run -- \
      python3 bench.py ${A[$TRACE]} --inflight 1 --no-profile > gpurun_out/${TAG}_${TRACE}_prof.log 2>&1
  rc=$?; echo "$TRACE rocprof rc=$rc"
  if [ $rc -eq 139 ] && ls gpurun_out/${TAG}_${TRACE}_prof/*kernel_stats.csv > /dev/null 2>&1; then
    echo "$TRACE: rocprofv3's exit-time segfault after the stats were written (cooperative launch)"; exit 0
  fi
  exit $rc
fi
