cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "export or dicom or montage or shot" > gpurun_out/r3x2_tests.log 2>&1 || { tail -20 gpurun_out/r3x2_tests.log; exit 1; }
tail -1 gpurun_out/r3x2_tests.log
