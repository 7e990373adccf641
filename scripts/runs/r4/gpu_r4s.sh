#!/bin/bash
# GPU-box (round 4): host-to-host with the 512-thread study build (two studies per CU) and large
# sub-batches, against the 1024-thread default at 224 x 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4s}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run t1024_s224x3 python scripts/h2h_leg.py --sub 224 --slots 3 --batches 12
for cfg in "448 2" "480 2" "512 2" "448 3" "384 3" "256 3"; do
  set -- $cfg
  VH_LIB_PATH=$PWD/scratch_libs/tpb512.so run t512_s${1}x${2} python scripts/h2h_leg.py --sub $1 --slots $2 --batches 12
done
VH_LIB_PATH=$PWD/scratch_libs/tpb512.so run t512_b512_inf2 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-h2h --batch 480 --inflight 2
for f in gpurun_out/${TAG}_*.json; do python3 -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d.get('vol_s', d.get('value')), d.get('runs_seconds'))"; done
