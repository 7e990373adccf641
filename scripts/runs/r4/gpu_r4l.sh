#!/bin/bash
# GPU-box (round 4): the 1024-thread default with the 70 KB layout -- the whole -m gpu suite, then
# the default bench (h2h with the link probe).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4l}
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r4l_bench.json") if l.startswith("{")][-1])
r = d["roofline"]
print(d["value"], d["ms_per_step"], d["batch_latency_ms"], d["n4_study_times"], r.get("frac"), r.get("isolated"))
print("h2h", d["host_to_host_vol_s"], d["host_to_host"].get("link"))
print("cpu", d["cpu_baseline"])
PY
