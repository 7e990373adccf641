#!/bin/bash
# GPU-box: config 5 at fixed iteration counts (--conv-threshold 0) for the default library and
# scratch_libs/ variants (LIBS), kernel classes per launch (A/B of kernel builds at constant work)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
for lib in default $LIBS default; do
  if [ $lib = default ]; then L=vent_analysis_amd/libventhip.so; else L=scratch_libs/$lib.so; fi
  VH_LIB_PATH=$L timeout -k 10 400 python3 bench.py --shape 512 512 512 --batch 1 --morph3d --steps 1 --warmup 1 --inflight 1 \
      --iso-runs 1 --conv-threshold 0 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_$lib.json 2> gpurun_out/${TAG}_$lib.err
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -3 gpurun_out/${TAG}_$lib.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; k=r['kernel_us_per_launch']; print(sys.argv[2], d['ms_per_step'], 'fit', k.get('n4_fit'), 'den', k.get('n4_den'), 'eval', k.get('n4_eval'), 'pcg', k.get('n4_pcg'))" gpurun_out/${TAG}_$lib.json $lib
done
