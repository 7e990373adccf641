# H2D ordering: none / device-side / host-side, on one box (after a PCIe probe)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pipe" > gpurun_out/r3ho_tests.log 2>&1 || { tail -3 gpurun_out/r3ho_tests.log; exit 1; }
tail -1 gpurun_out/r3ho_tests.log
timeout -k 10 120 python3 scripts/dev/h2h_probe.py > gpurun_out/r3ho_probe.log 2>&1; tail -2 gpurun_out/r3ho_probe.log
for rep in 1 2; do
for o in 1 2 0; do
  VH_PIPE_H2D_ORDER=$o timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3ho_$o.json 2> gpurun_out/r3ho_$o.err || exit 4
  python3 -c "import json;d=json.loads(open('gpurun_out/r3ho_$o.json').read());print('order=$o', d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
done
done
