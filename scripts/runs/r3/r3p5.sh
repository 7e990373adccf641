# host-to-host sweep on one box: sub-batch x slots (lag default)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "128 4" "128 6" "128 5" "64 8" "96 6" "128 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3p5_$1_$2.json 2> gpurun_out/r3p5_$1_$2.err || exit 4
  python3 -c "import json;d=json.loads(open('gpurun_out/r3p5_$1_$2.json').read());print('$1 $2', d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
done
