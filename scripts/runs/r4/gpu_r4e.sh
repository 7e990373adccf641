#!/bin/bash
# GPU-box (round 4): the study kernel at 512 threads (8 waves per study, one study per CU: how much
# slower is a study on half the waves?), its study-driver parity tests, the CI line, and the
# emap series probes (ST_PROF, study 3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4e}
run() { local name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err;
        local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run base1 python bench.py --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-h2h
VH_LIB_PATH=$PWD/scratch_libs/tpb512.so run tpb512 python bench.py --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-h2h
VH_LIB_PATH=$PWD/scratch_libs/tpb512.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py -k "study or bench_workload" > gpurun_out/${TAG}_tpb512_tests.log 2>&1
rc=$?; echo "tpb512 tests rc=$rc"; tail -2 gpurun_out/${TAG}_tpb512_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pipe" > gpurun_out/${TAG}_pipe_tests.log 2>&1
rc=$?; echo "pipe tests rc=$rc"; tail -2 gpurun_out/${TAG}_pipe_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  run h2h_new_$i python scripts/h2h_leg.py
  VH_PIPE_H2D_ORDER=1 VH_PIPE_D2H_LATE=0 run h2h_old_$i python scripts/h2h_leg.py
done
VH_PIPE_TRACE=1 run h2h_trace python scripts/h2h_leg.py
run ci python bench.py --workload ci --steps 20 --warmup 3
VH_LIB_PATH=$PWD/scratch_libs/stprof_b3.so run stprof_b3 python bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-h2h
grep ST_PROF gpurun_out/${TAG}_stprof_b3.json
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4e_*.json")):
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception:
        continue
    if "vol_s" in d:
        print(os.path.basename(f), "h2h", d["vol_s"], d["runs_seconds"]); continue
    r = d.get("roofline") or {}
    print(os.path.basename(f), d["value"], d.get("n4_study_times"), (r.get("kernel_ms_per_step") or {}).get("n4_study"),
          d.get("config", {}).get("cases") and {k: (v["seconds_per_map"], v["ci_walk_us"]) for k, v in d["config"]["cases"].items()})
PY
