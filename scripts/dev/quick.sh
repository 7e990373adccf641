#!/bin/bash
# GPU-box dev loop: a parity subset (K), then bench kernel times for each VH_PS_XS in XS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
K=${K:-"plane_sweep or snr or chain or border or batch or morph3d or empty or config or n4_vs"}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "$K" > gpurun_out/q_tests.log 2>&1
rc=$?; tail -1 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
for xs in ${XS:-32}; do
  VH_PS_XS=$xs timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2h > gpurun_out/q_bench_$xs.json 2> gpurun_out/q_bench_$xs.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -3 gpurun_out/q_bench_$xs.err; exit $rc; }
  python3 -c "import json;d=json.loads(open('gpurun_out/q_bench_$xs.json').read().strip().splitlines()[-1]);print('XS=$xs', d['value'], d['roofline']['kernel_ms_per_step'])"
done
