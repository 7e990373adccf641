#!/bin/bash
# GPU-box: everything the round's evidence needs, in order, stopping at the first failure:
# GPU parity suite, smoke, bench (with CPU baseline), rocprofv3 kernel stats, PMC traffic passes.
# usage: scripts/gpu_round.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -1 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-h2h > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
REGEX='k_n4_|k_tile|k_gather|k_snr|k_sort_vol|k_mask_stats' bash scripts/gpu_pmc.sh ${TAG}
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/${TAG}_traffic.json profiles/${TAG}_pmc_traffic.json
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json; exit $rc
