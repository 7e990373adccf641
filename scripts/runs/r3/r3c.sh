cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "n4 or bench_workload or config or kmeans or ci_ or recon" > gpurun_out/r3c_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r3c_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || exit 2
python3 -c "import json;d=json.loads(open('gpurun_out/r3c_bench.json').read());print(d['value'], d['roofline']['kernel_ms_per_step']['n4_study'], d['n4_study_times'])"
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3c_pcprof.log 2>&1 || exit 3
grep -c PCW_PROF gpurun_out/r3c_pcprof.log
