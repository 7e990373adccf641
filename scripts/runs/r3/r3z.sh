# round-3 evidence, part B: PMC traffic passes, per-study wall times, config lines
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_pmc.sh r3z_pmc || exit 1
cat gpurun_out/r3z_pmc_summary.log | tail -5
timeout -k 10 200 python scripts/study_times.py gpurun_out/r3z_study_times.json > gpurun_out/r3z_study_times.log 2>&1 || exit 2
head -2 gpurun_out/r3z_study_times.log
PROF="ci comm1" bash scripts/gpu_lines.sh r3z || exit 3
exit 0
