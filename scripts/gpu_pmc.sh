#!/bin/bash
# GPU-box: PMC counter passes (one rocprofv3 run per pass, counters only -- no trace domains) on a
# short bench.  Default: the FETCH_SIZE and WRITE_SIZE passes for roofline.traffic, summarised by
# scripts/pmc_summary.py into gpurun_out/${TAG}_traffic.json.  PASSES overrides the pass list
# (";"-separated), REGEX the kernel filter, BENCH_ARGS the workload (default: the default bench's
# shape and batch, one batch at a time); the summary records it (bench.workload_key).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
REGEX=${REGEX:-k_n4_|k_tile|k_gather|k_snr}
IFS=';' read -ra LIST <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE}"
dirs=()
i=0
for PASS in "${LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PASS --kernel-include-regex "$REGEX" --output-format csv \
      -d gpurun_out/${TAG}_p$i -o pmc -- python3 bench.py --steps 2 --warmup 1 --inflight 1 --iso-runs 1 --no-cpu-baseline --no-profile --no-h2h $BENCH_ARGS \
      > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i ($PASS) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  dirs+=(gpurun_out/${TAG}_p$i)
done
if [ -z "$PASSES" ]; then
  BENCH_ARGS="$BENCH_ARGS" python3 scripts/pmc_summary.py gpurun_out/${TAG}_traffic.json "${dirs[@]}" > gpurun_out/${TAG}_summary.log 2>&1
fi
