# restructured pipe slots: parity tests, then host-to-host (traced and not)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "pipe or host or class" > gpurun_out/r3p6_tests.log 2>&1 || { tail -5 gpurun_out/r3p6_tests.log; exit 1; }
tail -1 gpurun_out/r3p6_tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3p6_h2h$i.json 2> gpurun_out/r3p6_h2h$i.err || exit 4
python3 -c "import json;d=json.loads(open('gpurun_out/r3p6_h2h$i.json').read());print(d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
done
VH_PIPE_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3p6_h2ht.json 2> gpurun_out/r3p6_h2ht.err || exit 5
python3 -c "import json;d=json.loads(open('gpurun_out/r3p6_h2ht.json').read());print(d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
