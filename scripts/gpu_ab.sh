#!/bin/bash
# GPU-box: A/B benchmark of library variants under scratch_libs/ (VH_LIB_PATH), one bench each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-$(cd scratch_libs && ls *.so | sed 's/\.so$//')}; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['value'], d['roofline']['kernel_ms_per_step'])"
done
