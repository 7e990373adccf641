# host-to-host right after the full GPU suite vs a second process later (traced both)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r3q2_pytest.log 2>&1 || { tail -3 gpurun_out/r3q2_pytest.log; exit 1; }
tail -1 gpurun_out/r3q2_pytest.log
for i in 1 2; do
VH_PIPE_TRACE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3q2_h2h$i.json 2> gpurun_out/r3q2_h2h$i.err || exit 4
python3 -c "import json;d=json.loads(open('gpurun_out/r3q2_h2h$i.json').read());print($i, d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
done
free -g | head -2
