cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3s3_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r3s3_smoke.log; exit $rc
