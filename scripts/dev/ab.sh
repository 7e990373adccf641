#!/bin/bash
# GPU-box: bench kernel times for each scratch_libs/*.so variant (VARIANTS="a b" to choose)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-$(cd scratch_libs && ls *.so | sed 's/\.so$//')}; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-h2h ${BENCH_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -3 gpurun_out/ab_$v.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);k=d['roofline']['kernel_ms_per_step'];print('$v', d['value'], {n: k[n] for n in k if n != 'n4_study'}, 'study', k.get('n4_study'))"
done
