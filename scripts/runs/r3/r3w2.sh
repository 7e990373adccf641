# ST_EVAL_EXP A/B: eval stores exp(d); parity of the variant, then bench both builds twice
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
VH_LIB_PATH=$PWD/scratch_libs/eexp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "n4 or bench or vdp or batch" > gpurun_out/r3w2_tests.log 2>&1 || { tail -5 gpurun_out/r3w2_tests.log; exit 1; }
tail -1 gpurun_out/r3w2_tests.log
for rep in 1 2; do
for v in base eexp; do
  if [ $v = base ]; then unset VH_LIB_PATH; else export VH_LIB_PATH=$PWD/scratch_libs/eexp.so; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3w2_$v.json 2> gpurun_out/r3w2_$v.err || exit 3
  python3 -c "import json;d=json.loads(open('gpurun_out/r3w2_$v.json').read());print('$v', d['value'], d['roofline']['kernel_ms_per_step']['n4_study'])"
done
done
