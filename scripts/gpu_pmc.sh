#!/bin/bash
# GPU-box: PMC counter passes (one rocprofv3 run per pass, counters only -- no trace domains) on a
# short bench, restricted to the N4 sweep kernels and the classify kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
REGEX=${REGEX:-k_n4_eval|k_n4_fit|k_n4_hist|k_tile}
i=0
for PASS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
            ${EXTRA_PASS:+"$EXTRA_PASS"}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PASS --kernel-include-regex "$REGEX" --output-format csv \
      -d gpurun_out/${TAG}_p$i -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile \
      > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
