"""Phase timeline of the per-particle map merge (k_map_merge) from a -DESLAM_STAMPS build:
    ESLAM_GPU_LIB=$PWD/slam-eslam_amd/lib/ab/lib_stamps.so python tools/stamps_maps.py [particles] [warmup] [patches]
The bench's configs[4] workload (bench.py --local-maps): `warmup` steps with a map update each,
then one more whose merge is stamped (the first particle group of each of the first 32768
blocks).  Read the shares, not the lengths: the stamps' waits slow the build."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import eslam_abi as A  # noqa: E402
import eslam_amd  # noqa: E402
import synthetic as S  # noqa: E402
from stamps import report  # noqa: E402

MG_PHASES = ["start", "record + codes", "first stage landed", "first stage applied", "passes done", "counted"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 * 1024 * 1024
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    patches = int(sys.argv[3]) if len(sys.argv) > 3 else 48
    L = eslam_amd.load_library()
    L.eslam_gpu_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_uint64]
    L.eslam_gpu_debug_stamps.restype = C.c_int64
    grid = S.unmapped_beyond(S.rough_map(), 0.3)
    scan = S.scan_area(patches) if patches != 48 else S.scan_patches()
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    cfg.local_map_pages = 0 if patches <= 64 else 40
    f = eslam_amd.GpuFilter(cfg, device=0)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    steps = S.step_stream(warm + 1, tilt=True)
    for st in steps[:-1]:
        f.step(st)
        f.map_update(scan)
    f.step(steps[-1])
    f.sync()
    assert L.eslam_gpu_debug_stamps_clear() == 0
    f.map_update(scan)
    f.sync()
    buf = np.zeros((32768, 8), dtype=np.uint64)
    blocks = L.eslam_gpu_debug_stamps(5, buf.ctypes.data, 32768)
    assert blocks >= 0
    report(f"k_map_merge at n={n}, {patches} patches ({blocks} blocks launched)", buf.copy(), MG_PHASES, min(blocks, 32768))
    f.close()


if __name__ == "__main__":
    main()
