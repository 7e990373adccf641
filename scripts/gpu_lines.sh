#!/bin/bash
# GPU-box: the per-config perf lines besides the default bench: config 2
# (256x256x24, batch 1, sweep driver), config 5 (512^3, batch 1, 3-D morphology), the CI line
# (defect-voxels/s), and the RCCL path at --gpus 1 (--comm).  Benches first, then rocprofv3 kernel
# stats for the lines named in PROF (default "ci comm1 config2").  config 2 goes last: its
# cooperative launch (grid PC) still makes rocprofv3 itself segfault at exit (rc 139 after the
# statistics are written; DESIGN.md section 9, profiles/r3i_exit_fault.txt): a 139 with the stats
# CSV present counts as that line done, and nothing more runs on the GPU after it.
# usage: [LINES="config2 ci"] [PROF="ci comm1"] scripts/gpu_lines.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
declare -A ARGS
ARGS[config2]="--shape 256 256 24 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-h2h"
ARGS[config5]="--shape 512 512 512 --batch 1 --morph3d --steps 2 --warmup 1 --no-cpu-baseline --no-h2h"
ARGS[ci]="--workload ci --steps 20 --warmup 3"
ARGS[comm1]="--comm --steps 5 --warmup 1 --no-cpu-baseline --no-h2h"
LINES=${LINES-config2 config5 ci comm1}
PROF=${PROF-ci comm1 config2}
for name in $LINES; do
  timeout -k 10 600 python3 bench.py ${ARGS[$name]} > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${name}.err; exit $rc; }
done
for name in $PROF; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${name}_prof -o run -- \
      python3 bench.py ${ARGS[$name]} --no-profile > gpurun_out/${TAG}_${name}_prof.log 2>&1
  rc=$?; echo "$name rocprof rc=$rc"
  if [ $rc -eq 139 ] && ls gpurun_out/${TAG}_${name}_prof/*kernel_stats.csv > /dev/null 2>&1; then
    echo "$name: rocprofv3's exit-time segfault after the stats were written; stopping here"; exit 0
  fi
  [ $rc -eq 0 ] || exit $rc
done
