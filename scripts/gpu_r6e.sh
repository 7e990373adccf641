#!/bin/bash
# round-6 step: grid tests with the tagged-granule PC records, then the phase profile and the one-study
# lines (A/B: records through grid barriers, VH_STG_BARRIER_PC=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6e}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "grid or config2 or n4_vs_oracle" > gpurun_out/${TAG}_grid_tests.log 2>&1
rc=$?; echo "grid tests rc=$rc"; tail -2 gpurun_out/${TAG}_grid_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_stgprof.sh $TAG stgprof || exit 1
grep STG_PROF gpurun_out/${TAG}_stgprof_*.log | tail -4
for ab in 0 1; do
  VH_STG_BARRIER_PC=$ab MODES=grid INFL="1 3" SKIP_SUITE=1 bash scripts/gpu_grid_check_lines.sh ${TAG}_b$ab || exit 1
done
