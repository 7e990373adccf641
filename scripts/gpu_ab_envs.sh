#!/bin/bash
# GPU-box: the default bench under several environment settings, alternated twice; prints value,
# step and every class's time per step.  usage: scripts/gpu_ab_envs.sh TAG "A-settings" "B-settings" ...
# ("-" = no setting; a setting is "VAR=VALUE [VAR2=VALUE2 ...]")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
for round in 1 2; do
  i=0
  for set in "$@"; do
    i=$((i + 1))
    if [ "$set" = - ]; then E=(); else E=($set); fi
    env "${E[@]}" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h \
        > gpurun_out/${TAG}_${i}_$round.json 2> gpurun_out/${TAG}_${i}_$round.err
    rc=$?; [ $rc -eq 0 ] || { echo "$set rc=$rc"; tail -3 gpurun_out/${TAG}_${i}_$round.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], 'lat', d.get('batch_latency_ms'), 'non_n4', r.get('non_n4_us_per_step'), 'wall', r.get('non_n4_wall_us_per_step'), {k: v for k, v in r['kernel_us_per_step'].items() if k != 'n4_study'})" gpurun_out/${TAG}_${i}_$round.json "$set"
  done
done
