#!/bin/bash
# GPU-box (round 4): batches in flight with more hardware queues per process (GPU_MAX_HW_QUEUES 8:
# one queue per batch stream, so no two batches' kernels serialise on a shared queue).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4j}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-h2h"
GPU_MAX_HW_QUEUES=8 VH_STUDY_TRACE=gpurun_out/${TAG}_q8_inf4.csv run q8_inf4 $B --inflight 4
GPU_MAX_HW_QUEUES=8 run q8_inf3 $B --inflight 3
GPU_MAX_HW_QUEUES=8 run q8_inf6 $B --inflight 6
GPU_MAX_HW_QUEUES=8 VH_LIB_PATH=$PWD/scratch_libs/tpb1024.so run q8_t1024_inf3 $B --inflight 3
GPU_MAX_HW_QUEUES=8 VH_LIB_PATH=$PWD/scratch_libs/tpb1024.so run q8_t1024_inf4 $B --inflight 4
echo "== q8_inf4"; python3 scripts/study_trace.py gpurun_out/${TAG}_q8_inf4.csv
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4j_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(os.path.basename(f), d["value"], d.get("batch_latency_ms"), d.get("n4_study_times"))
PY
