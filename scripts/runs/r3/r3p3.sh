# same box: PCIe probe (incl. both directions at once), then host-to-host direct vs staged
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/dev/h2h_probe.py > gpurun_out/r3p3_probe.log 2>&1 || { cat gpurun_out/r3p3_probe.log; exit 1; }
cat gpurun_out/r3p3_probe.log
for st in 0 1; do
  if [ $st = 1 ]; then export VH_PIPE_STAGE=1; fi
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3p3_h2h_$st.json 2> gpurun_out/r3p3_h2h_$st.err || exit 4
  python3 -c "import json;d=json.loads(open('gpurun_out/r3p3_h2h_$st.json').read());print('stage=$st', d['value'], d['host_to_host_vol_s'], d['host_to_host']['runs_seconds'])"
done
