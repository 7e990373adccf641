#!/bin/bash
# GPU-box: the -m gpu suite with scratch_libs/$NEW.so, then config 2 / config 5 lines alternated
# between $OLD and $NEW builds.  usage: OLD=rc1 NEW=sw1 scripts/dev/gpu_cfg_ab.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=${1:-cfg}
VH_LIB_PATH=$PWD/scratch_libs/$NEW.so timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in $OLD $NEW; do
    for c in config2 config5; do
      if [ $c = config2 ]; then A="--shape 256 256 24 --batch 1 --steps 10 --warmup 2"; else A="--shape 512 512 512 --batch 1 --morph3d --steps 2 --warmup 1"; fi
      VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 300 python bench.py $A --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_${v}_${c}_$r.json 2> gpurun_out/${TAG}_${v}_${c}_$r.err
      rc=$?; [ $rc -eq 0 ] || { echo "$v $c rc=$rc"; tail -3 gpurun_out/${TAG}_${v}_${c}_$r.err; exit $rc; }
      python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${v}_${c}_$r.json').read().splitlines()[-1]);print('$v $c $r', d['value'], d['unit'], d['ms_per_step'])"
    done
  done
done
