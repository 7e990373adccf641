#!/bin/bash
# GPU-box: per-phase cycle counts of k_n4_study (ST_PROF variants under scratch_libs/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-$(cd scratch_libs && ls *.so | sed 's/\.so$//')}; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --n4-mode study ${BENCH_ARGS} > gpurun_out/phase_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -3 gpurun_out/phase_$v.log; exit $rc; }
  echo "$v $(grep -E "ST_PROF|CH_PROF" gpurun_out/phase_$v.log | tail -2 | tr "\n" " ") | $(python3 -c "import json;d=json.loads(open('gpurun_out/phase_$v.log').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['kernel_ms_per_step'].get('n4_study'))")"
done
