cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh tests || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_k1c.log 2>&1 || exit 1
bash tools/pmc.sh k1c --steps 5 --warmup 2 > gpurun_out/pmc_k1c.txt 2>&1
