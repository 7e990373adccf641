# isolate the r3q fault: the class-shim test alone (no pipe run before it), then pipe + class shim,
# then the whole suite + bench and the traced h2h runs
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "class_shim_matches" > gpurun_out/r3r_t1.log 2>&1 || { tail -5 gpurun_out/r3r_t1.log; exit 1; }
timeout -k 10 300 $T tests/test_gpu_parity.py -k "pipe_host_to_host_equals_batch or class_shim_matches" > gpurun_out/r3r_t2.log 2>&1 || { tail -5 gpurun_out/r3r_t2.log; exit 2; }
bash scripts/gpu_suite.sh r3r || exit 3
bash scripts/dev/r3p.sh || exit 4
exit 0
