#!/bin/bash
# GPU-box: the default bench with the tree's library (A) and scratch_libs/ variants, alternated
# twice (A V1 V2 ... A V1 V2 ...); prints value, step, the isolated study launch and every class's
# time per step.  usage: scripts/gpu_ab_libs.sh TAG VARIANT [VARIANT ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
for round in 1 2; do
  for v in A "$@"; do
    if [ $v = A ]; then L=vent_analysis_amd/libventhip.so; else L=scratch_libs/$v.so; fi
    VH_LIB_PATH=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h \
        > gpurun_out/${TAG}_${v}_$round.json 2> gpurun_out/${TAG}_${v}_$round.err
    rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/${TAG}_${v}_$round.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], 'iso', r['avg_launch_us'], 'non_n4', r.get('non_n4_us_per_step'), {k: v for k, v in r['kernel_us_per_step'].items() if k != 'n4_study'})" gpurun_out/${TAG}_${v}_$round.json $v
  done
done
