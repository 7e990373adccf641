# host-to-host timelines over the bench's three passes (default 128 x 4)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
VH_PIPE_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3p2_h2h.json 2> gpurun_out/r3p2_h2h.err || exit 4
python3 -c "import json;d=json.loads(open('gpurun_out/r3p2_h2h.json').read());print(d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
nproc; numactl -H 2>/dev/null | head -3; cat /proc/cpuinfo | grep "model name" | head -1
