# branch-free eval / fit row groups (prefetch effective): GPU suite + bench, then the traced h2h runs
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_suite.sh r3q || exit 1
bash scripts/dev/r3p.sh || exit 2
exit 0
