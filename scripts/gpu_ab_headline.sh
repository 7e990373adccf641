#!/bin/bash
# GPU-box: the default bench alternated between the tree's library and a scratch_libs/ variant
# (A B A B), no CPU baseline / host-to-host; prints value and the isolated k_n4_study launch.
# usage: scripts/gpu_ab_headline.sh TAG LIB_B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; B=$2
for lib in A B A B; do
  if [ $lib = A ]; then L=vent_analysis_amd/libventhip.so; else L=scratch_libs/$B.so; fi
  VH_LIB_PATH=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h \
      > gpurun_out/${TAG}_$lib.json 2> gpurun_out/${TAG}_$lib.err
  rc=$?; [ $rc -eq 0 ] || { echo "$lib rc=$rc"; tail -3 gpurun_out/${TAG}_$lib.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], 'iso', r['avg_launch_us'], 'study mean', d['n4_study_times']['mean_us'], 'sort', r['kernel_us_per_launch'].get('sort'), 'non_n4', r.get('non_n4_us_per_step'))" gpurun_out/${TAG}_$lib.json $lib
done
