# GPU suite + bench (certified early convergence decision), PC + phase profiles, h2h direct vs staged
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh r3l || exit 1
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3l_pcprof.log 2>&1 || exit 2
grep -c "xsig 1" gpurun_out/r3l_pcprof.log; grep -c PCW_PROF gpurun_out/r3l_pcprof.log
VH_LIB_PATH=$PWD/scratch_libs/stp.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3l_stprof.log 2>&1 || exit 3
grep ST_PROF gpurun_out/r3l_stprof.log | tail -2
timeout -k 10 200 python scripts/study_times.py gpurun_out/r3l_study_times.json > gpurun_out/r3l_study_times.log 2>&1 || exit 4
head -2 gpurun_out/r3l_study_times.log
exit 0
