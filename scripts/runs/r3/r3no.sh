cd $GRAFT_REPO_ROOT
bash scripts/dev/r3o.sh || exit 1
bash scripts/dev/r3n.sh || exit 2
