#!/bin/bash
# GPU-box: k_n4_study's traffic split by phase: FETCH_SIZE / WRITE_SIZE passes at
# fixed iteration counts (--conv-threshold 0: 4 x 50 iterations per study) with S7 by PC (conv_mode
# 0) and without it (conv_mode 1, the exact CoV from item sums: no d, no PC): the difference is PC's.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
for cm in 0 1; do
  REGEX='k_n4_study' BENCH_ARGS="--conv-threshold 0 --conv-mode $cm" bash scripts/gpu_pmc.sh ${TAG}_cm$cm || exit 1
  cat gpurun_out/${TAG}_cm${cm}_summary.log
done
