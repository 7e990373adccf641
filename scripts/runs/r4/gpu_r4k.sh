#!/bin/bash
# GPU-box (round 4): stream priorities for batches in flight (VH_PRIO=1: the study kernel on a
# low-priority stream, every other kernel of the batch high), 512 and 1024 threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4k}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-h2h"
VH_PRIO=1 VH_STUDY_TRACE=gpurun_out/${TAG}_p_inf2.csv run p_inf2 $B --inflight 2
VH_PRIO=1 run p_inf3 $B --inflight 3
GPU_MAX_HW_QUEUES=8 VH_PRIO=1 run p_q8_inf4 $B --inflight 4
VH_PRIO=1 VH_LIB_PATH=$PWD/scratch_libs/tpb1024.so run p_t1024_inf2 $B --inflight 2
VH_PRIO=1 VH_LIB_PATH=$PWD/scratch_libs/tpb1024.so run p_t1024_inf3 $B --inflight 3
run base_inf2 $B --inflight 2
echo "== p_inf2"; python3 scripts/study_trace.py gpurun_out/${TAG}_p_inf2.csv
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4k_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(os.path.basename(f), d["value"], d.get("batch_latency_ms"), d.get("n4_study_times"))
PY
