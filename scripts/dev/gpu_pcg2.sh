#!/bin/bash
# GPU-box: the grid-PC parity tests, then config 2 / config 5 lines (default build) and the PCG_PROF round counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pcg2}
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "config2 or config5 or rerun_bit or pc_equals_serial" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
LINES="config2 config5" PROF="" bash scripts/gpu_lines.sh ${TAG}
rc=$?; [ $rc -eq 0 ] || exit $rc
for c in config2 config5; do python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_$c.json').read().splitlines()[-1]);r=d['roofline'];print('$c', d['value'], d['ms_per_step'], r['kernel_us_per_launch'])"; done
bash scripts/dev/prof_pcg.sh ${TAG}p
