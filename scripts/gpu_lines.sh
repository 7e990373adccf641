#!/bin/bash
# GPU-box: the per-config perf lines besides the default bench, each with its
# rocprofv3 kernel stats: config 2 (256x256x24, batch 1, sweep driver), config 5 (512^3, batch 1,
# 3-D morphology), the CI line (defect-voxels/s), and the RCCL path at --gpus 1 (--comm).
# usage: scripts/gpu_lines.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
run() {   # name, timeout, bench args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python3 bench.py "$@" > gpurun_out/${TAG}_${name}.json 2> gpurun_out/${TAG}_${name}.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_${name}.err; exit $rc; }
  timeout -k 10 $to rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${name}_prof -o run -- \
      python3 bench.py "$@" --no-profile > gpurun_out/${TAG}_${name}_prof.log 2>&1
  rc=$?; echo "$name rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run config2 300 --shape 256 256 24 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-h2h
run config5 600 --shape 512 512 512 --batch 1 --morph3d --steps 2 --warmup 1 --no-cpu-baseline --no-h2h
run ci 300 --workload ci --steps 20 --warmup 3
run comm1 300 --comm --steps 5 --warmup 1 --no-cpu-baseline --no-h2h
