# expf_fast in PC pass 0: parity suite subset (N4 / PC), then the PC profile and a bench line
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "n4 or pc or vdp or bench or config" > gpurun_out/r3x_tests.log 2>&1 || { tail -5 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3x_pcprof.log 2>&1 || exit 2
grep PCW_PROF gpurun_out/r3x_pcprof.log | head -3
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3x_bench.json 2> gpurun_out/r3x_bench.err || exit 3
python3 -c "import json;d=json.loads(open('gpurun_out/r3x_bench.json').read());print(d['value'], d['roofline']['kernel_ms_per_step']['n4_study'])"
for v in stp stpu; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3x_$v.log 2>&1 || exit 4
  echo $v; grep ST_PROF gpurun_out/r3x_$v.log | tail -2
done
