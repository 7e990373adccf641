cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
VH_LIB_PATH=$PWD/scratch_libs/stp.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3w_stprof.log 2>&1 || exit 1
grep ST_PROF gpurun_out/r3w_stprof.log | tail -4
