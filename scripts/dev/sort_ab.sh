cd $GRAFT_REPO_ROOT
for v in s_hist s_p1; do VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$v.json 2>&1 || exit 1; python3 -c "import json;d=json.loads(open('gpurun_out/$v.json').read().strip().splitlines()[-1]);print('$v', d['roofline']['kernel_ms_per_step'].get('sort'))"; done
