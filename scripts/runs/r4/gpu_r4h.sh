#!/bin/bash
# GPU-box (round 4): where the 512-thread study workgroups run (VH_STUDY_TRACE): one launch of
# 512 studies, and two 256-study batches in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4h}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-h2h"
VH_STUDY_TRACE=gpurun_out/${TAG}_b512.csv run b512 $B --inflight 1 --batch 512
VH_STUDY_TRACE=gpurun_out/${TAG}_inf2.csv run inf2 $B --inflight 2
VH_STUDY_TRACE=gpurun_out/${TAG}_b512_one.csv VH_ST_MIN_LDS=90000 run b512_one $B --inflight 1 --batch 512
for f in b512 inf2 b512_one; do echo "== $f"; python3 scripts/study_trace.py gpurun_out/${TAG}_$f.csv; done
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4h_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(os.path.basename(f), d["value"], d.get("n4_study_times"))
PY
