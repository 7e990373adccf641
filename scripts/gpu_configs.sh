#!/bin/bash
# GPU-box: the config-2 / config-5 lines with their own PMC traffic.  Per config:
# FETCH_SIZE / WRITE_SIZE passes of that workload (the summary records the library's sha256 and the
# workload, copied into the box's profiles/ so the line reads it), then the bench line.  Last, one
# rocprofv3 kernel trace (TRACE=config2|config5): its cooperative grid-PC launch makes rocprofv3
# itself segfault at exit after the statistics are written (rc 139), so it is
# the call's final GPU step and nothing runs after it.
# NOTE: a --pmc pass of a workload with a cooperative launch (configs 2 and 5) ends in that same
# exit-time segfault (r6a: counters written, rc 139), so PMC passes of those configs go one per call
# (scripts/gpu_pmc1.sh); NOPMC=1 skips them here.
# usage: [NOPMC=1] [CONFIGS="config2 config5"] [TRACE=config5] scripts/gpu_configs.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
declare -A WL STEPS
WL[config2]="--shape 256 256 24 --batch 1"
WL[config5]="--shape 512 512 512 --batch 1 --morph3d"
WL[one]="--shape 128 128 24 --batch 1"
STEPS[config2]="--steps 10 --warmup 2"
STEPS[config5]="--steps 3 --warmup 1"
STEPS[one]="--steps 20 --warmup 3"
for c in ${CONFIGS-config2 config5}; do
  if [ -z "$NOPMC" ]; then
  REGEX='k_n4_|k_plane|k_sort|k_kmeans' BENCH_ARGS="${WL[$c]}" bash scripts/gpu_pmc.sh ${TAG}_${c}_pmc
  rc=$?; echo "$c pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/${TAG}_${c}_pmc_traffic.json profiles/${TAG}_${c}_pmc_traffic.json
  fi
  timeout -k 10 600 python3 bench.py ${WL[$c]} ${STEPS[$c]} --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_${c}.json 2> gpurun_out/${TAG}_${c}.err
  rc=$?; echo "$c bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${c}.err; exit $rc; }
done
if [ -n "${TRACE-config5}" ]; then
  c=${TRACE-config5}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${c}_prof -o run -- \
      python3 bench.py ${WL[$c]} ${STEPS[$c]} --inflight 1 --no-cpu-baseline --no-h2h --no-profile > gpurun_out/${TAG}_${c}_prof.log 2>&1
  rc=$?; echo "$c rocprof rc=$rc"
  if [ $rc -eq 139 ] && ls gpurun_out/${TAG}_${c}_prof/*kernel_stats.csv > /dev/null 2>&1; then
    echo "$c: rocprofv3's exit-time segfault after the stats were written (cooperative launch)"; exit 0
  fi
  exit $rc
fi
