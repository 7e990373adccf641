# GPU suite + bench (PCX walks from prefetched registers, pipe DMA from registered caller buffers),
# PC profile, h2h with staging forced (A/B)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh r3k || exit 1
VH_LIB_PATH=$PWD/scratch_libs/pcp.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-h2h > gpurun_out/r3k_pcprof.log 2>&1 || exit 2
grep PCW_X gpurun_out/r3k_pcprof.log | head -6
for cfg in "128 4" "256 3"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3k_h2h_$1_$2.json 2> gpurun_out/r3k_h2h_$1_$2.err || exit 4
  VH_PIPE_STAGE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --h2h-sub $1 --h2h-slots $2 > gpurun_out/r3k_h2hs_$1_$2.json 2> gpurun_out/r3k_h2hs_$1_$2.err || exit 5
  python3 -c "import json;d=json.loads(open('gpurun_out/r3k_h2h_$1_$2.json').read());e=json.loads(open('gpurun_out/r3k_h2hs_$1_$2.json').read());print('$1 $2 direct', d['value'], d['host_to_host_vol_s'], 'staged', e['value'], e['host_to_host_vol_s'])"
done
# SQ counters of the study kernel (one pass, counters only)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-include-regex "k_n4_study" --output-format csv -d gpurun_out/r3k_sq -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-h2h > gpurun_out/r3k_sq.log 2>&1
echo "sq pass rc=$?"
exit 0
