cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/d1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py::test_zero_measurement_variance_stops_the_update tests/test_parity_lineage.py > gpurun_out/d1/pytest.log 2>&1; echo pytest rc=$?
L=$PWD/slam-eslam_amd/lib/libeslam_gpu_eslam_k1_prof.so
N=262144 ESLAM_GPU_LIB=$L timeout -k 10 120 python tools/k1_prof.py > gpurun_out/d1/regions_256k.log 2>&1 &&
N=4194304 ESLAM_GPU_LIB=$L timeout -k 10 120 python tools/k1_prof.py > gpurun_out/d1/regions_4m.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d1/t256 -o run -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 --particles 262144 > gpurun_out/d1/t256.log 2>&1
