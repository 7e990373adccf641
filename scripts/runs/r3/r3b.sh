cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/study_times.py gpurun_out/r3b_study_times.json > gpurun_out/r3b_study_times.log 2>&1 || exit 1
head -3 gpurun_out/r3b_study_times.log
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3b_pcprof.log 2>&1 || exit 2
grep -c PCW_PROF gpurun_out/r3b_pcprof.log
VH_LIB_PATH=$PWD/scratch_libs/stp.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3b_stprof.log 2>&1 || exit 3
grep ST_PROF gpurun_out/r3b_stprof.log | tail -2
