#!/bin/bash
# round-6 step: grid-PC pass 0 through the LDS transpose (sweep driver): parity tests, then config 5
# A/B (VH_PCG_T0=0 the round-5 pass 0), config 2 on the sweeps likewise
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6g}
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "config5 or pc_equals or sweep or config2 or class_pooled" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for ab in 1 0 1 0; do
  VH_PCG_T0=$ab timeout -k 10 400 python3 bench.py --shape 512 512 512 --batch 1 --morph3d --steps 3 --warmup 1 --inflight 1 \
      --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_c5_t$ab.json 2> gpurun_out/${TAG}_c5_t$ab.err
  rc=$?; [ $rc -eq 0 ] || { echo "c5 rc=$rc"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print('config5 T0', sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_us'], r['kernel_us_per_step']['n4_pcg'])" gpurun_out/${TAG}_c5_t$ab.json $ab
done
timeout -k 10 200 python3 bench.py --workload class --steps 20 --warmup 3 > gpurun_out/${TAG}_class.json 2> gpurun_out/${TAG}_class.err
rc=$?; echo "class rc=$rc"; cat gpurun_out/${TAG}_class.json
