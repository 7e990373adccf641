cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pipe" > gpurun_out/r3t2_tests.log 2>&1 || { tail -30 gpurun_out/r3t2_tests.log; exit 1; }
grep -c PASSED gpurun_out/r3t2_tests.log; tail -1 gpurun_out/r3t2_tests.log
