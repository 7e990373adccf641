#!/bin/bash
# GPU-box: config 5 alternated between the tree's library and scratch_libs/LIB_B (default convergence)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; B=$2
for lib in A B A B; do
  if [ $lib = A ]; then L=vent_analysis_amd/libventhip.so; else L=scratch_libs/$B.so; fi
  VH_LIB_PATH=$L timeout -k 10 400 python3 bench.py --shape 512 512 512 --batch 1 --morph3d --steps 3 --warmup 1 --inflight 1 \
      --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_$lib.json 2> gpurun_out/${TAG}_$lib.err
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -3 gpurun_out/${TAG}_$lib.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], 'pcg', r['kernel_us_per_launch'].get('n4_pcg'))" gpurun_out/${TAG}_$lib.json $lib
done
