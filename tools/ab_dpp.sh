cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -2 gpurun_out/ab/pytest.log
bash tools/ab_run.sh 3 slam-eslam_amd/lib/libeslam_gpu_base.so slam-eslam_amd/lib/libeslam_gpu.so > gpurun_out/ab/ab4m.log 2>&1 || exit 1
BENCH_ARGS="--particles 262144" bash tools/ab_run.sh 3 slam-eslam_amd/lib/libeslam_gpu_base.so slam-eslam_amd/lib/libeslam_gpu.so > gpurun_out/ab/ab256k.log 2>&1
cat gpurun_out/ab/ab4m.log gpurun_out/ab/ab256k.log
