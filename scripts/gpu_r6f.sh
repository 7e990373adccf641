#!/bin/bash
# round-6 step: the grid form's workgroup count on config 2; config 5 with the (1-2^-24)^m decision
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6f}
for G in 12 16 24 32 48; do
  VH_STG_G=$G timeout -k 10 200 python3 bench.py --shape 256 256 24 --batch 1 --steps 10 --warmup 2 --inflight 1 \
      --no-cpu-baseline --no-h2h --n4-mode grid > gpurun_out/${TAG}_c2_G$G.json 2> gpurun_out/${TAG}_c2_G$G.err
  rc=$?; [ $rc -eq 0 ] || { echo "G $G rc=$rc"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('G', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_c2_G$G.json $G
done
timeout -k 10 400 python3 bench.py --shape 512 512 512 --batch 1 --morph3d --steps 3 --warmup 1 --inflight 1 \
    --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_config5.json 2> gpurun_out/${TAG}_config5.err
rc=$?; echo "config5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print('config5', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['frac'], r['kernel_us_per_step'])" gpurun_out/${TAG}_config5.json
VH_LIB_PATH=scratch_libs/pcgprof.so timeout -k 10 400 python3 bench.py --shape 512 512 512 --batch 1 --morph3d --steps 1 --warmup 0 \
    --inflight 1 --iso-runs 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_config5_pcgprof.log 2>&1
rc=$?; echo "config5 pcgprof rc=$rc"; grep -c "decided" gpurun_out/${TAG}_config5_pcgprof.log; grep -c "PCG2" gpurun_out/${TAG}_config5_pcgprof.log
exit $rc
