#!/bin/bash
# GPU-box (round 4): why the 512-thread / 70 KB study kernel is slower per study (r4f).  A/B of
# one vs two studies per CU on the same build (VH_ST_MIN_LDS pads the dynamic LDS past 80 KB), the
# same layout at 1024 threads, and ST_PROF phase splits of study 3 in both placements.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4g}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h"
VH_ST_MIN_LDS=90000 run one_inf1 $B --inflight 1
VH_ST_MIN_LDS=90000 run one_inf2 $B --inflight 2
VH_LIB_PATH=$PWD/scratch_libs/tpb1024.so run t1024_inf1 $B --inflight 1
VH_LIB_PATH=$PWD/scratch_libs/tpb1024.so run t1024_inf2 $B --inflight 2
VH_LIB_PATH=$PWD/scratch_libs/stprof_b3.so run prof_two python bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-h2h
VH_ST_MIN_LDS=90000 VH_LIB_PATH=$PWD/scratch_libs/stprof_b3.so run prof_one python bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-h2h
grep -h ST_PROF gpurun_out/${TAG}_prof_two.json gpurun_out/${TAG}_prof_one.json
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4g_*.json")):
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception:
        continue
    r = d.get("roofline") or {}
    print(os.path.basename(f), d["value"], d.get("batch_latency_ms"), d.get("n4_study_times"),
          (r.get("kernel_ms_per_step") or {}).get("n4_study"))
PY
