# per-study N4 wall times, PC / study-kernel phase profiles, host-to-host sweep (sub-batch x slots)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r3g}
timeout -k 10 200 python scripts/study_times.py gpurun_out/${T}_study_times.json > gpurun_out/${T}_study_times.log 2>&1 || exit 1
head -3 gpurun_out/${T}_study_times.log
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/${T}_pcprof.log 2>&1 || exit 2
grep -c PCW_PROF gpurun_out/${T}_pcprof.log
VH_LIB_PATH=$PWD/scratch_libs/stp.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/${T}_stprof.log 2>&1 || exit 3
grep ST_PROF gpurun_out/${T}_stprof.log | tail -2
for cfg in "64 6" "32 8" "128 4" "256 3"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/${T}_h2h_$1_$2.json 2> gpurun_out/${T}_h2h_$1_$2.err || exit 4
  python3 -c "import json;d=json.loads(open('gpurun_out/${T}_h2h_$1_$2.json').read());print('$1 $2', d['value'], d['host_to_host_vol_s'])"
done
