# GPU suite + bench (current build), A/B bench against scratch_libs/base.so, then r3g's profiles
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh r3f || exit 1
VH_LIB_PATH=$PWD/scratch_libs/base.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h2h > gpurun_out/r3f_base.json 2> gpurun_out/r3f_base.err || exit 2
python3 -c "import json;d=json.loads(open('gpurun_out/r3f_base.json').read());print('base', d['value'], d['roofline']['kernel_ms_per_step']['n4_study'])"
TAG=r3f bash scripts/dev/r3g.sh
