# host-to-host pipeline sweep (sub-batch size x slots) and the per-config lines
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "256 3" "64 6" "32 8" "128 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3e_h2h_$1_$2.json 2> gpurun_out/r3e_h2h_$1_$2.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r3e_h2h_$1_$2.json').read());print('$1 $2', d['value'], d['host_to_host_vol_s'])"
done
timeout -k 10 1200 bash scripts/gpu_lines.sh r3e
