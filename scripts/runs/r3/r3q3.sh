# copy-ordering A/B on one box (after the GPU suite, as the driver's order): H2D order x late D2H
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "pipe" > gpurun_out/r3q3_pytest.log 2>&1 || { tail -3 gpurun_out/r3q3_pytest.log; exit 1; }
tail -1 gpurun_out/r3q3_pytest.log
timeout -k 10 120 python3 scripts/dev/h2h_probe.py > gpurun_out/r3q3_probe.log 2>&1; tail -2 gpurun_out/r3q3_probe.log
for rep in 1 2; do
for v in "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  VH_PIPE_H2D_ORDER=$1 VH_PIPE_D2H_LATE=$2 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3q3_$1$2.json 2> gpurun_out/r3q3_$1$2.err || exit 4
  python3 -c "import json;d=json.loads(open('gpurun_out/r3q3_$1$2.json').read());print('order=$1 late=$2', d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
done
done
