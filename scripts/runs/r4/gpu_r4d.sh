#!/bin/bash
# GPU-box (round 4): batches in flight 1/2/3 with the largest-first study order, and the
# host-to-host leg after a device-resident warm-up / a CPU load (the bench's order) vs cold.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4d}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run bench python bench.py --steps 20 --warmup 5
run inflight1 python bench.py --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-h2h
run inflight3 python bench.py --steps 21 --warmup 6 --inflight 3 --no-cpu-baseline --no-h2h
run inflight4 python bench.py --steps 20 --warmup 8 --inflight 4 --no-cpu-baseline --no-h2h
run h2h_cold python scripts/h2h_leg.py
run h2h_warm python scripts/h2h_leg.py --warm-device 25
run h2h_cpu python scripts/h2h_leg.py --cpu-load 15
run h2h_cold2 python scripts/h2h_leg.py
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4d_*.json")):
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception:
        continue
    if "vol_s" in d:
        print(os.path.basename(f), "h2h", d["vol_s"], d["runs_seconds"])
    else:
        r = d.get("roofline") or {}
        print(os.path.basename(f), d["value"], "lat", d.get("batch_latency_ms"), "h2h", d.get("host_to_host_vol_s"),
              "frac", r.get("frac"), "iso", r.get("isolated"), (r.get("kernel_ms_per_step") or {}).get("n4_study"))
PY
