#!/bin/bash
# GPU-box: why host-to-host trails device-resident.  The default bench line,
# then the host-to-host leg alone: A/B with the device batch held open (round-3 bench) or not,
# a VH_PIPE_TRACE timeline, and a rocprofv3 kernel + memory-copy trace (copies as SDMA records or
# as __amd_rocclr_copyBuffer blit kernels).  usage: scripts/gpu_h2h.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-h2h}
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for kb in "" "--unaligned"; do
    timeout -k 10 120 python scripts/h2h_leg.py $kb >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "h2h_leg $kb rc=$rc"; exit $rc; }
  done
done
cat gpurun_out/${TAG}_ab.jsonl | python -c "import sys,json; [print('aligned', d['aligned'], d['vol_s'], d['runs_seconds']) for d in map(json.loads, sys.stdin)]"
VH_PIPE_TRACE=1 timeout -k 10 120 python scripts/h2h_leg.py > gpurun_out/${TAG}_trace.json 2> gpurun_out/${TAG}_pipe_trace.txt
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d gpurun_out/${TAG}_prof -o run -- python3 scripts/h2h_leg.py > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
