#!/bin/bash
# GPU-box (round 4): bench with one / two batches in flight, sort-chunk A/B, per-study phase
# profiles of studies 1 and 3, and the host-to-host leg's dependence on torch's runtime init and
# on the late D2H enqueue.  usage: scripts/gpu_r4c.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4c}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run bench python bench.py --steps 20 --warmup 5
run inflight2 python bench.py --steps 20 --warmup 5 --inflight 2 --no-cpu-baseline --no-h2h
run inflight3 python bench.py --steps 21 --warmup 6 --inflight 3 --no-cpu-baseline --no-h2h
for v in base kpt16; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so run ab_$v python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h
done
for v in stprof_b1 stprof_b3; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so run $v python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h
done
for i in 1 2; do
  run h2h_plain_$i python scripts/h2h_leg.py
  run h2h_torch_$i python scripts/h2h_leg.py --torch
  VH_PIPE_D2H_LATE=1 run h2h_late_$i python scripts/h2h_leg.py
  VH_PIPE_D2H_LATE=1 run h2h_torch_late_$i python scripts/h2h_leg.py --torch
done
python3 - <<'PY'
import json, glob, os
tag = os.environ.get("TAG", "r4c")
for f in sorted(glob.glob(f"gpurun_out/*_*.json")):
    if "r4c_" not in f: continue
    try:
        ln = [l for l in open(f) if l.startswith("{")][-1]
        d = json.loads(ln)
    except Exception as e:
        continue
    if "vol_s" in d:
        print(os.path.basename(f), "h2h", d["vol_s"], d["runs_seconds"])
    elif "value" in d:
        r = d.get("roofline") or {}
        print(os.path.basename(f), d["value"], d.get("batch_latency_ms"), (r.get("kernel_ms_per_step") or {}))
PY
