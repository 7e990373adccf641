# fix4 (non-returning limb atomics) in the sweep driver's fit: N4 parity (sweep driver, large, config 5), config 5 timing
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "n4 or large or config5 or pc or ragged or grid" > gpurun_out/r3u2_tests.log 2>&1 || { tail -5 gpurun_out/r3u2_tests.log; exit 1; }
tail -1 gpurun_out/r3u2_tests.log
A="--shape 512 512 512 --batch 1 --morph3d --steps 2 --warmup 1 --no-cpu-baseline --no-h2h"
timeout -k 10 300 python3 bench.py $A --no-profile > gpurun_out/r3u2_c5np.json 2> gpurun_out/r3u2_c5np.err || exit 2
timeout -k 10 300 python3 bench.py $A > gpurun_out/r3u2_c5.json 2> gpurun_out/r3u2_c5.err || exit 3
timeout -k 10 300 python3 bench.py --shape 256 256 24 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3u2_c2.json 2> gpurun_out/r3u2_c2.err || exit 4
python3 -c "
import json;d=json.loads(open('gpurun_out/r3u2_c5np.json').read());e=json.loads(open('gpurun_out/r3u2_c5.json').read());c=json.loads(open('gpurun_out/r3u2_c2.json').read());print('c5 noprof', d['ms_per_step'], 'prof', e['ms_per_step'], 'c2', c['value']);k=e['roofline']['kernel_ms_per_step'];print(sorted(k.items(),key=lambda x:-x[1])[:6])"
