cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh testsall smoke bench benchsharded
