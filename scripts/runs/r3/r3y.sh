# round-3 evidence, part A: GPU suite + short bench, the default bench (CPU baseline, host-to-host),
# rocprofv3 kernel statistics of the bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh r3z || exit 1
timeout -k 10 900 python bench.py > gpurun_out/r3z_bench_full.json 2> gpurun_out/r3z_bench_full.err || exit 2
cat gpurun_out/r3z_bench_full.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3z_prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2h --no-profile > gpurun_out/r3z_prof.log 2>&1
echo "rocprof rc=$?"
exit 0
