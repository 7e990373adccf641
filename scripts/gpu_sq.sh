#!/bin/bash
# GPU-box: one rocprofv3 --pmc pass of SQ stall counters (8 SQ slots on gfx950, MI355X_MICROARCH.md)
# on the headline batch's k_n4_study, then on config 5's sweep kernels (the cooperative grid PC makes
# rocprofv3 segfault at exit after writing the counters, so that pass is the call's last step).
# usage: scripts/gpu_sq.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sq}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex 'k_n4_study' --output-format csv \
    -d gpurun_out/${TAG}_head -o pmc -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --iso-runs 1 \
    --no-cpu-baseline --no-profile --no-h2h > gpurun_out/${TAG}_head.log 2>&1
rc=$?; echo "headline sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-include-regex 'k_n4_pcg|k_n4_fit|k_n4_eval' --output-format csv \
    -d gpurun_out/${TAG}_c5 -o pmc -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --iso-runs 1 \
    --no-cpu-baseline --no-profile --no-h2h --shape 512 512 512 --batch 1 --morph3d > gpurun_out/${TAG}_c5.log 2>&1
rc=$?; echo "config5 sq rc=$rc"
if [ $rc -eq 139 ] && [ -s gpurun_out/${TAG}_c5/pmc_counter_collection.csv ]; then
  echo "rocprofv3's exit-time segfault after the counters were written (cooperative launch)"; exit 0
fi
exit $rc
