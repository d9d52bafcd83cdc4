cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/d3
python - > gpurun_out/d3/occ.log 2>&1 <<'PY'
import ctypes as C, sys
sys.path.insert(0, "slam-eslam_amd")
import eslam_amd
lib = eslam_amd.load_library()
occ = C.c_int(0)
for lds in (-1, 0, 36864):
    lib.eslam_debug_k1_occupancy(C.byref(occ), lds)
    print("normal build: dynamic LDS", lds, "blocks per CU", occ.value)
PY
L=$PWD/slam-eslam_amd/lib/libeslam_gpu_eslam_k1_tl.so
N=262144 ESLAM_GPU_LIB=$L timeout -k 10 120 python tools/k1_timeline.py > gpurun_out/d3/tl_256k.log 2>&1
cat gpurun_out/d3/*.log
