cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/d2
L=$PWD/slam-eslam_amd/lib/libeslam_gpu_eslam_k1_tl.so
N=262144 ESLAM_GPU_LIB=$L timeout -k 10 120 python tools/k1_timeline.py > gpurun_out/d2/tl_256k.log 2>&1 &&
N=4194304 ESLAM_GPU_LIB=$L timeout -k 10 120 python tools/k1_timeline.py > gpurun_out/d2/tl_4m.log 2>&1
cat gpurun_out/d2/tl_256k.log gpurun_out/d2/tl_4m.log
