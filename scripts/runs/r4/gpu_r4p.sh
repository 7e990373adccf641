#!/bin/bash
# GPU-box (round 4): CUs reserved for the batches' short kernels (VH_ST_RESERVE=k: the study kernel
# on a stream whose CU mask leaves k CUs per XCD free), device-resident and host-to-host.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4p}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-h2h"
run base_inf2 $B --inflight 2
VH_ST_RESERVE=1 VH_STUDY_TRACE=gpurun_out/${TAG}_r1_inf2.csv run r1_inf2 $B --inflight 2
VH_ST_RESERVE=1 run r1_inf3 $B --inflight 3
VH_ST_RESERVE=2 run r2_inf2 $B --inflight 2
VH_ST_RESERVE=2 run r2_inf3 $B --inflight 3
VH_ST_RESERVE=1 run h_r1_s256x3 python scripts/h2h_leg.py --sub 256 --slots 3 --batches 12
VH_ST_RESERVE=1 run h_r1_s224x3 python scripts/h2h_leg.py --sub 224 --slots 3 --batches 12
run h_s224x3 python scripts/h2h_leg.py --sub 224 --slots 3 --batches 12
echo "== r1_inf2"; python3 scripts/study_trace.py gpurun_out/${TAG}_r1_inf2.csv
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4p_*.json")):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    if "vol_s" in d:
        print(os.path.basename(f), "h2h", d["vol_s"], d["runs_seconds"]); continue
    print(os.path.basename(f), d["value"], d.get("batch_latency_ms"), d.get("n4_study_times"))
PY
