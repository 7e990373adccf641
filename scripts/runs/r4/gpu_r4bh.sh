#!/bin/bash
# GPU-box (round 4 evidence, FIT_G 6 on top of r4bc): the -m gpu suite, the default bench, rocprofv3
# kernel-trace statistics of the bench, the FETCH_SIZE / WRITE_SIZE passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4bh}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh ${TAG}_pmc
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cat gpurun_out/${TAG}_pmc_summary.log | head -12
python3 - <<'PY'
import json, csv, glob
d = json.loads([l for l in open("gpurun_out/r4bh_bench.json") if l.startswith("{")][-1])
r = d["roofline"]
print("bench", d["value"], d["ms_per_step"], d["batch_latency_ms"], d["n4_study_times"], r.get("frac"), r.get("isolated"))
print("h2h", d["host_to_host_vol_s"], d["host_to_host"].get("link"))
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["per_core_vol_s"])
rows = list(csv.DictReader(open(glob.glob("gpurun_out/r4bh_trace/*kernel_stats.csv")[0])))
for x in rows[:12]:
    print(x["Name"][:40], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), "us", x["Percentage"])
PY
