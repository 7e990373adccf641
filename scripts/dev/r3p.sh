# host-to-host pipeline timelines (VH_PIPE_TRACE) at two sub-batch / slot shapes
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "128 4" "256 2" "64 4"; do
  set -- $cfg
  VH_PIPE_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3p_h2h_$1_$2.json 2> gpurun_out/r3p_h2h_$1_$2.err || exit 4
  python3 -c "import json;d=json.loads(open('gpurun_out/r3p_h2h_$1_$2.json').read());print('$1 $2', d['value'], d['host_to_host_vol_s'])"
done
