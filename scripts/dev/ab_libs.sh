#!/bin/bash
# GPU-box A/B of scratch_libs/<name>.so variants: bench n4_study ms for each name given.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in "$@"; do VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h2h ${AB_ARGS} > gpurun_out/ab_$v.json 2>/dev/null || exit 1; python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline']['kernel_ms_per_step']['n4_study'])"; done
