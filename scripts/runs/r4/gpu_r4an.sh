#!/bin/bash
# GPU-box: the RCCL cohort all-reduce on the communicator's own stream (batches in flight issue it
# in program order): the one-rank RCCL test, then bench --comm with three batches in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4an}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "rccl or smoke" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "rccl test rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --comm --steps 20 --warmup 3 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_bench_comm.json 2> gpurun_out/${TAG}_bench_comm.err
rc=$?; echo "bench comm rc=$rc"; tail -c 600 gpurun_out/${TAG}_bench_comm.json; [ $rc -eq 0 ] || exit $rc
