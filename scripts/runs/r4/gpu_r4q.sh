#!/bin/bash
# GPU-box (round 4): the default bench with the new host-to-host defaults (224 x 3, 12 x 256 studies).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4q}
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r4q_bench.json") if l.startswith("{")][-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], d["batch_latency_ms"], d["n4_study_times"], r.get("frac"), r.get("isolated"))
print("h2h", d["host_to_host_vol_s"], d["host_to_host"].get("link"), d["host_to_host"]["runs_seconds"])
PY
