#!/bin/bash
# GPU-box (round 4): stage-0 rounds skip the steps of blocks certified frozen at their start -- study-driver parity,
# the per-study PC trace, the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4af}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "study or bench_workload or n4 or pc or sweep" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
VH_STUDY_TRACE=gpurun_out/${TAG}_trace.csv timeout -k 10 300 python bench.py --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_b1.json 2> gpurun_out/${TAG}_b1.err
rc=$?; echo "trace bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/study_pc.py gpurun_out/${TAG}_trace.csv
timeout -k 10 300 python bench.py --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json
for f in ("gpurun_out/r4af_b1.json", "gpurun_out/r4af_bench.json"):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, d["value"], d["ms_per_step"], d.get("batch_latency_ms"), d["n4_study_times"], (d["roofline"] or {}).get("isolated"))
PY
