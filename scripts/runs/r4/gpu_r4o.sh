#!/bin/bash
# GPU-box (round 4): host-to-host sweep over 12 x 256 studies (pipeline fill / drain amortised).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4o}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
for cfg in "128 4" "192 3" "256 2" "256 3" "160 3" "224 3" "192 4"; do
  set -- $cfg
  run s${1}x${2} python scripts/h2h_leg.py --sub $1 --slots $2 --batches 12
done
for f in gpurun_out/${TAG}_*.json; do python3 -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['vol_s'], d['runs_seconds'])"; done
