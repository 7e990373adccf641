# host-to-host: per-chunk pinning overlapped with compute, direct vs staged, sub-batch sweep
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "pipe or host" > gpurun_out/r3n_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r3n_tests.log; [ $rc -eq 0 ] || exit 1
for cfg in "128 4" "64 6" "256 3"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3n_h2h_$1_$2.json 2> gpurun_out/r3n_h2h_$1_$2.err || exit 4
  VH_PIPE_STAGE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3n_h2hs_$1_$2.json 2> gpurun_out/r3n_h2hs_$1_$2.err || exit 5
  python3 -c "import json;d=json.loads(open('gpurun_out/r3n_h2h_$1_$2.json').read());e=json.loads(open('gpurun_out/r3n_h2hs_$1_$2.json').read());print('$1 $2 direct', d['value'], d['host_to_host_vol_s'], 'staged', e['value'], e['host_to_host_vol_s'])"
done
