# per-config lines + rocprof stats, PMC traffic of the default bench, host-side pinning probe
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/dev/h2h_probe.py > gpurun_out/r3h_h2h_probe.log 2>&1; cat gpurun_out/r3h_h2h_probe.log
timeout -k 10 900 bash scripts/gpu_lines.sh r3h || exit 1
timeout -k 10 400 bash scripts/gpu_pmc.sh r3h_pmc || exit 2
cat gpurun_out/r3h_pmc_summary.log | tail -5
