#!/bin/bash
# GPU-box: PC round counts / cycles of block 0 per iteration (scratch_libs/pcp.so, a -DPC_PROF build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline --no-h2h > gpurun_out/pcprof.log 2>&1
rc=$?; grep -c PCW_PROF gpurun_out/pcprof.log; exit $rc
