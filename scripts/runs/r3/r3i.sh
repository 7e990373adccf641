# GPU suite + bench (PCX fast walks), PC profile, then the exit-time fault under rocprofv3:
# a minimal cooperative launch, config 2 with the grid PC off, config 2 with the maps dumped
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh r3i || exit 1
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3i_pcprof.log 2>&1 || exit 2
grep PCW_PROF gpurun_out/r3i_pcprof.log | head -3
for c in 0 1; do
  timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3i_coop$c -o run -- scripts/microbench/coop_exit $c > gpurun_out/r3i_coop$c.log 2>&1
  echo "coop_exit $c under rocprofv3: rc=$?"
done
VH_N4_PCG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3i_c2nopcg -o run -- python3 bench.py --shape 256 256 24 --batch 1 --steps 3 --warmup 1 --no-cpu-baseline --no-h2h --no-profile > gpurun_out/r3i_c2nopcg.log 2>&1
echo "config2 without k_n4_pcg under rocprofv3: rc=$?"
VH_DUMP_MAPS=gpurun_out/r3i_maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3i_c2 -o run -- python3 bench.py --shape 256 256 24 --batch 1 --steps 3 --warmup 1 --no-cpu-baseline --no-h2h --no-profile > gpurun_out/r3i_c2.log 2>&1
echo "config2 under rocprofv3 (maps dumped): rc=$?"
exit 0
