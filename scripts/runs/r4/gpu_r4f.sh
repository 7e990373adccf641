#!/bin/bash
# GPU-box (round 4): the study kernel at 512 threads and <= 80 KB of LDS (two studies per CU):
# study-driver parity first, then the bench at 1-3 batches in flight, then the whole -m gpu suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4f}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py -k "study or bench_workload" > gpurun_out/${TAG}_study_tests.log 2>&1
rc=$?; echo "study tests rc=$rc"; tail -3 gpurun_out/${TAG}_study_tests.log; [ $rc -eq 0 ] || exit $rc
VH_N4_DEBUG=1 run inflight1 python bench.py --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-h2h
grep "N4 study driver" gpurun_out/${TAG}_inflight1.err | sort | uniq -c
run inflight2 python bench.py --steps 10 --warmup 2 --inflight 2 --no-cpu-baseline --no-h2h
run inflight3 python bench.py --steps 10 --warmup 2 --inflight 3 --no-cpu-baseline --no-h2h
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4f_*.json")):
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception:
        continue
    r = d.get("roofline") or {}
    print(os.path.basename(f), d["value"], d.get("batch_latency_ms"), d.get("n4_study_times"),
          (r.get("kernel_ms_per_step") or {}).get("n4_study"), r.get("frac"), (r.get("isolated") or {}).get("avg_launch_us"))
PY
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log
