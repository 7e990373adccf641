# host-to-host pipeline timelines (VH_PIPE_TRACE) at several sub-batch / slot shapes; lag = default
# (chunks that fill the CUs) unless the third field sets VH_PIPE_LAG
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "128 4 d" "256 3 d" "128 4 0" "64 6 d" "128 3 d"; do
  set -- $cfg
  if [ "$3" = d ]; then unset VH_PIPE_LAG; else export VH_PIPE_LAG=$3; fi
  VH_PIPE_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3p_h2h_$1_$2_$3.json 2> gpurun_out/r3p_h2h_$1_$2_$3.err || exit 4
  python3 -c "import json;d=json.loads(open('gpurun_out/r3p_h2h_$1_$2_$3.json').read());print('$1 $2 $3', d['value'], d['host_to_host_vol_s'])"
done
