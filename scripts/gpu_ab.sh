#!/bin/bash
# GPU-box: alternated A/B of library variants (VH_LIB_PATH; "base" = the in-tree libventhip.so),
# REPS rounds over VARIANTS (base | a scratch_libs/NAME.so build | VAR=VALUE), one short bench each: the isolated k_n4_study launch (mean of 5 runs of
# one batch alone) and the device-resident rate.  usage: VARIANTS="base apx3" REPS=2 scripts/gpu_ab.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-ab}
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base}; do
    # a variant is "base" (the in-tree library), a scratch_libs/NAME.so build, or VAR=VALUE (an
    # environment setting with the in-tree library)
    lib=$PWD/vent_analysis_amd/libventhip.so; envs=""
    case "$v" in base) ;; *=*) envs="$v" ;; *) lib=$PWD/scratch_libs/$v.so ;; esac
    env VH_LIB_PATH=$lib $envs timeout -k 10 200 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --no-h2h ${BENCH_ARGS} \
        > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err
    rc=$?; [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; tail -3 gpurun_out/${TAG}_${v}_$r.err; exit $rc; }
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${v}_$r.json').read().splitlines()[-1]);r=d['roofline'];k=r['kernel_us_per_launch'];print('$v', $r, d['value'], r['avg_launch_us'], r['kernel'], d['n4_study_times'], {n: k[n] for n in k if n != 'n4_study'}, 'non_n4', r.get('non_n4_us_per_step'))"
  done
done
