# k_n4_hred: large-volume tests, then the config 5 line without event timers
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "config5 or large or pc_grid or grid or 256" > gpurun_out/r3u_tests.log 2>&1 || { tail -5 gpurun_out/r3u_tests.log; exit 1; }
tail -2 gpurun_out/r3u_tests.log
A="--shape 512 512 512 --batch 1 --morph3d --steps 2 --warmup 1 --no-cpu-baseline --no-h2h"
timeout -k 10 300 python3 bench.py $A --no-profile > gpurun_out/r3u_c5np.json 2> gpurun_out/r3u_c5np.err || exit 2
timeout -k 10 300 python3 bench.py $A > gpurun_out/r3u_c5.json 2> gpurun_out/r3u_c5.err || exit 3
python3 -c "
import json;d=json.loads(open('gpurun_out/r3u_c5np.json').read());e=json.loads(open('gpurun_out/r3u_c5.json').read());print('noprof', d['ms_per_step'], 'prof', e['ms_per_step']);k=e['roofline']['kernel_ms_per_step'];print(sorted(k.items(),key=lambda x:-x[1])[:8])"
