# final build check: GPU suite + default bench (device-resident, CPU baseline, host-to-host)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r3zz_pytest_gpu.log 2>&1 || { tail -5 gpurun_out/r3zz_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3zz_pytest_gpu.log
timeout -k 10 900 python bench.py > gpurun_out/r3zz_bench.json 2> gpurun_out/r3zz_bench.err || exit 2
python3 -c "import json;d=json.loads(open('gpurun_out/r3zz_bench.json').read());print(d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'], d['cpu_baseline']['value'], d['roofline']['frac'], d['roofline']['traffic_source'])"
