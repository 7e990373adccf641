# fit ring depth sensitivity (ST_PROF): FIT_NB 4 (default) vs 2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in stp stp2; do
  VH_LIB_PATH=$PWD/scratch_libs/$v.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3nb_$v.log 2>&1 || exit 1
  echo $v; grep ST_PROF gpurun_out/r3nb_$v.log | tail -2
done
