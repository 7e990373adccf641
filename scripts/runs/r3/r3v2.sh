cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3v2_pcprof.log 2>&1 || exit 2
grep PCW_P0 gpurun_out/r3v2_pcprof.log | head -5; grep -c PCW_P0 gpurun_out/r3v2_pcprof.log
