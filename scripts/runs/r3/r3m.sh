# bench + phase profile (fit loads one group ahead)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "n4 or bench_workload" > gpurun_out/r3m_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r3m_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3m_bench.json 2> gpurun_out/r3m_bench.err || exit 2
python3 -c "import json;d=json.loads(open('gpurun_out/r3m_bench.json').read());print(d['value'], d['roofline']['kernel_ms_per_step']['n4_study'], d['n4_study_times'])"
VH_LIB_PATH=$PWD/scratch_libs/stp2.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3m_stprof.log 2>&1 || exit 3
grep ST_PROF gpurun_out/r3m_stprof.log | tail -2
