#!/bin/bash
# GPU-box: a round's evidence for the headline line, in order, stopping at the first failure:
#   smoke -> -m gpu suite -> FETCH_SIZE / WRITE_SIZE passes (the summary records the library's
#   sha256; bench.py uses its traffic only for the same build) -> rocprofv3 kernel-trace statistics
#   of one batch at a time (the isolated launch durations the bench's roofline uses) -> bench.py
#   (default line with the CPU baseline and host-to-host).  Only gpurun_out/ comes back from the
#   box; the PMC summary is also copied into the box's profiles/ so this run's bench reads it.
# usage: scripts/gpu_evidence.sh TAG [SKIP_SUITE=1]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
REGEX='k_n4_|k_plane|k_gather|k_snr|k_sort_vol|k_mask_stats|k_kmeans' bash scripts/gpu_pmc.sh ${TAG}_pmc
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_traffic.json   # gpu_pmc.sh TAG_pmc -> TAG_pmc_traffic.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
    python3 bench.py --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-h2h --no-profile > gpurun_out/${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/evidence_check.py gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_trace/*kernel_stats.csv
