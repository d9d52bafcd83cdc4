cd $GRAFT_REPO_ROOT
bash tools/profile.sh r01c --steps 20 --warmup 5 > gpurun_out/profile_r01c.txt 2>&1 || exit 1
bash tools/pmc.sh r01c --steps 5 --warmup 2 > gpurun_out/pmc_r01c.txt 2>&1
