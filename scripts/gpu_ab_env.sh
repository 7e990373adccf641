#!/bin/bash
# GPU-box: the -m gpu suite (one process), then the default bench alternated between the tree's
# library as built (A) and the same library with an environment variable set (B), A B A B; prints
# value, step, the isolated study launch and the non-N4 classes.
# usage: scripts/gpu_ab_env.sh TAG "VAR=VALUE [VAR2=VALUE2 ...]" [pytest -k expr | all | none]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; ENVB=$2; K=${3:-all}
if [ "$K" != none ]; then
  if [ "$K" = all ]; then KARG=(); else KARG=(-k "$K"); fi
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ "${KARG[@]}" > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for v in A B A B; do
  if [ $v = A ]; then E=(); else E=($ENVB); fi
  env "${E[@]}" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h \
      > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/${TAG}_$v.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], 'iso', r['avg_launch_us'], 'non_n4', r.get('non_n4_us_per_step'), {k: v for k, v in r['kernel_us_per_step'].items() if k != 'n4_study'})" gpurun_out/${TAG}_$v.json $v
done
