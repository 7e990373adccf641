mkdir -p gpurun_out; export TMPDIR=/tmp
VH_LIB_PATH=$PWD/scratch_libs/stprof.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --inflight 1 --iso-runs 1 --no-cpu-baseline --no-h2h > gpurun_out/r5b_stprof.json 2> gpurun_out/r5b_stprof.err; rc=$?; echo "stprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
VH_LIB_PATH=$PWD/scratch_libs/pcprof.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --inflight 1 --iso-runs 1 --no-cpu-baseline --no-h2h > gpurun_out/r5b_pcprof.json 2> gpurun_out/r5b_pcprof.err; rc=$?; echo "pcprof rc=$rc"; exit $rc
