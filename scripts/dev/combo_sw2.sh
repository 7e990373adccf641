cd $GRAFT_REPO_ROOT
bash scripts/gpu_sweep_pc.sh sw2 || exit 1
bash scripts/dev/ab_sys2.sh
