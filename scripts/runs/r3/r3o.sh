# A/B at fixed work (4 x 50 iterations): current build vs eval without L0 loads, eval without stores,
# fit without U loads (results meaningless in B-D; only the kernel time is read)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in abA abB abC abD abA; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-h2h --conv-threshold 0 > gpurun_out/r3o_$v.json 2> gpurun_out/r3o_$v.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3o_$v.json').read());print('$v', d['value'], d['roofline']['kernel_ms_per_step']['n4_study'], d['n4_study_times']['mean_us'])"
done
