#!/bin/bash
# GPU-box (round 4): feeding two study slots per CU -- batches in flight at 512 threads (placement
# traces), 512-study batches in flight (the fed upper bound), 1024 threads at 3 in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4i}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-h2h"
VH_STUDY_TRACE=gpurun_out/${TAG}_inf3.csv run inf3 $B --inflight 3
VH_STUDY_TRACE=gpurun_out/${TAG}_inf4.csv run inf4 $B --inflight 4
run b512_inf2 $B --inflight 2 --batch 512
run b128_inf4 $B --inflight 4 --batch 128
VH_LIB_PATH=$PWD/scratch_libs/tpb1024.so run t1024_inf3 $B --inflight 3
for f in inf3 inf4; do echo "== $f"; python3 scripts/study_trace.py gpurun_out/${TAG}_$f.csv; done
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4i_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(os.path.basename(f), d["value"], d.get("batch_latency_ms"), d.get("n4_study_times"))
PY
