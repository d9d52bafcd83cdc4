# K3a/K3b tile size sweep: ESLAM_SCAN_ITEMS x particle counts (bench kernel_ms per variant)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/items
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_dist.py > gpurun_out/items/pytest.log 2>&1 || { tail -30 gpurun_out/items/pytest.log; exit 1; }
tail -2 gpurun_out/items/pytest.log
for n in 262144 1048576 4194304 16777216; do
  for it in 2 4 8 2 4 8; do
    printf "n=%s items=%s " $n $it
    ESLAM_SCAN_ITEMS=$it timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --particles $n | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])" || exit 1
  done
done 2>&1 | tee gpurun_out/items/sweep.log
