# fit ring rows in the free P1 buffer: N4 parity, fit profile, bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "n4 or bench or vdp or batch or ragged or pipe" > gpurun_out/r3rg_tests.log 2>&1 || { tail -5 gpurun_out/r3rg_tests.log; exit 1; }
tail -1 gpurun_out/r3rg_tests.log
VH_LIB_PATH=$PWD/scratch_libs/stp.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3rg_stprof.log 2>&1 || exit 2
grep ST_PROF gpurun_out/r3rg_stprof.log | tail -2
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3rg_bench$i.json 2> gpurun_out/r3rg_bench$i.err || exit 3
python3 -c "import json;d=json.loads(open('gpurun_out/r3rg_bench$i.json').read());print(d['value'], d['roofline']['kernel_ms_per_step']['n4_study'])"
done
