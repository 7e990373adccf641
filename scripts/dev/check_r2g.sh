cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "config or pc_equals or sweep or rerun or deterministic" > gpurun_out/r2g_tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -1 gpurun_out/r2g_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/het.json 2>gpurun_out/het.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/het.json').read().strip().splitlines()[-1]);print('het', d['value'], d['ms_per_step'], d['config']['n4_iterations_mean'], d['roofline']['kernel_ms_per_step']['n4_study'], d['host_to_host_vol_s'])"
timeout -k 10 300 python3 bench.py --shape 512 512 512 --batch 1 --morph3d --steps 2 --warmup 1 --no-cpu-baseline --no-h2h > gpurun_out/r2g_config5.json 2>/dev/null || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/r2g_config5.json').read().strip().splitlines()[-1]);print('c5', d['value'], d['ms_per_step'], list(d['roofline']['kernel_ms_per_step'].items())[:6])"
