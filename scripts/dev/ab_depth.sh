#!/bin/bash
# GPU-box A/B: study-kernel speculation depth / chain slots (scratch_libs/{d1,ns2,ns3}.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
VH_LIB_PATH=$PWD/scratch_libs/ns2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "study" > gpurun_out/ns2_tests.log 2>&1; echo "ns2 tests rc=$?"; tail -1 gpurun_out/ns2_tests.log
for v in d1 ns3 ns2; do VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2h > gpurun_out/ab_$v.json 2>/dev/null || exit 1; python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline']['kernel_ms_per_step']['n4_study'])"; done
