#!/bin/bash
# GPU-box: k-means parity subset, then alternated bench A/B of k_kmeans_s vs k_kmeans (VH_KM_OLD=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "kmeans or adversarial or class or vdp or degenerate or three" > gpurun_out/km_pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/km_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for old in 0 1; do
    VH_KM_OLD=$old timeout -k 10 200 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-h2h ${BENCH_ARGS} \
        > gpurun_out/km_${old}_$r.json 2> gpurun_out/km_${old}_$r.err
    rc=$?; [ $rc -eq 0 ] || { echo "old=$old rc=$rc"; tail -3 gpurun_out/km_${old}_$r.err; exit $rc; }
    python3 -c "import json;d=json.loads(open('gpurun_out/km_${old}_$r.json').read().splitlines()[-1]);r=d['roofline'];k=r['kernel_us_per_launch'];print('old=$old', d['value'], 'kmeans', k.get('kmeans'), 'sort', k.get('sort'), 'non_n4', r.get('non_n4_us_per_step'))"
  done
done
