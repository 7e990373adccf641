# scheduler-strategy A/B of the whole library (bench only; a kept variant gets the parity suite)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for v in base silp smem; do
  if [ $v = base ]; then unset VH_LIB_PATH; else export VH_LIB_PATH=$PWD/scratch_libs/$v.so; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3sched_$v.json 2> gpurun_out/r3sched_$v.err || exit 3
  python3 -c "import json;d=json.loads(open('gpurun_out/r3sched_$v.json').read());print('$v', d['value'], d['roofline']['kernel_ms_per_step']['n4_study'])"
done
done
