#!/bin/bash
# GPU-box (round 4): host-to-host sub-batch / slot sweep (the pipe at 128 x 4 behaves like 128-study
# batches in flight, which run 7.1 k vol/s device-resident, r4i).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4n}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run s128x4 python scripts/h2h_leg.py --sub 128 --slots 4
run s256x2 python scripts/h2h_leg.py --sub 256 --slots 2
run s256x3 python scripts/h2h_leg.py --sub 256 --slots 3
run s256x4 python scripts/h2h_leg.py --sub 256 --slots 4
run s192x3 python scripts/h2h_leg.py --sub 192 --slots 3
GPU_MAX_HW_QUEUES=8 run q8_s256x4 python scripts/h2h_leg.py --sub 256 --slots 4
GPU_MAX_HW_QUEUES=8 run q8_s128x6 python scripts/h2h_leg.py --sub 128 --slots 6
for f in gpurun_out/${TAG}_*.json; do python3 -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['vol_s'], d['runs_seconds'], d.get('pinned_peak_bytes'), d.get('staged_spans'))"; done
