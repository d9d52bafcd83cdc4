cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh tests || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench_k3c.log 2>&1
