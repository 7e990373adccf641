#!/bin/bash
# GPU-box: the sweep driver with PC (k_n4_pcw): sweep / config parity tests, then the config-2 and
# config-5 bench lines.  usage: scripts/gpu_sweep_pc.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sw}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sweep or config or deterministic" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --shape 256 256 24 --batch 1 --steps 5 --warmup 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_config2.json 2> gpurun_out/${TAG}_config2.err
rc=$?; echo "config2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_config2.json').read().strip().splitlines()[-1]);print('config2', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
timeout -k 10 400 python bench.py --shape 512 512 512 --batch 1 --morph3d --steps 1 --warmup 1 --no-cpu-baseline --no-h2h > gpurun_out/${TAG}_config5.json 2> gpurun_out/${TAG}_config5.err
rc=$?; echo "config5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_config5.json').read().strip().splitlines()[-1]);print('config5', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_step'])"
