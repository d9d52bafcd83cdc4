"""K1 per-wave timeline (diagnostic build with -DESLAM_K1_TL): when waves start, stage the
LDS window, load their first row, finish their rows, flush and exit, relative to the first
wave's entry (s_memrealtime, 100 MHz).

    python slam-eslam_amd/build_lib.py -DESLAM_K1_TL
    N=262144 ESLAM_GPU_LIB=slam-eslam_amd/lib/libeslam_gpu_eslam_k1_tl.so python tools/k1_timeline.py
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, "slam-eslam_amd")
sys.path.insert(0, "tests")
import eslam_abi as A  # noqa: E402
import eslam_amd  # noqa: E402
import synthetic as S  # noqa: E402

n = int(os.environ.get("N", 262144))
cfg = S.bench_config(A.default_config(), n)
f = eslam_amd.GpuFilter(cfg)
f.set_map(S.flat_map(cells=1000))
f.init_gaussian(n, [0, 0, 0], [0.1, 0.1, 0.1], 0.18, 1.001)
for st in S.step_stream(12):
    f.step(st)
f.sync()
lib = eslam_amd.load_library()
buf = (C.c_ulonglong * (8192 * 8))()
assert lib.eslam_debug_k1_tl(buf) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
waves = min(8192, (n + 63) // 64)
t = t[:waves]
t0 = t[:, 0].min()
names = ["entry", "staged", "-", "-", "-", "exit"]
print(f"n={n} waves={waves}  (us after the first wave's entry: min / median / max)")
for k, nm in enumerate(names):
    if nm == "-":
        continue
    v = (t[:, k] - t0) / 100.0
    print(f"{nm:12s} {v.min():7.2f} {np.median(v):7.2f} {v.max():7.2f}")
ent = (t[:, 0] - t0) / 100.0
hist, edges = np.histogram(ent, bins=[0, 1, 2, 4, 8, 16, 32, 64, 128, 256, 1e9])
print("entry histogram (us):", list(zip(edges[:-1].tolist(), hist.tolist())))
occ = C.c_int(0)
for lds in (-1, 0, 16384, 32768, 36864, 38912, 39936, 40448, 40960):
    lib.eslam_debug_k1_occupancy(C.byref(occ), lds)
    print("occupancy API: dynamic LDS", lds, "blocks per CU", occ.value)
try:
    import torch
    p = torch.cuda.get_device_properties(0)
except RuntimeError:
    p = None
if p is not None:
    print("shared mem per MP:", getattr(p, "shared_memory_per_multiprocessor", None), "per block:", getattr(p, "shared_memory_per_block", None),
      "regs per MP:", getattr(p, "regs_per_multiprocessor", None), "MPs:", p.multi_processor_count)
for a, b in ((0, 1), (1, 5), (0, 5)):  # noqa: E305
    d = (t[:, b] - t[:, a]) / 100.0
    print(f"{names[a]:>12s} -> {names[b]:12s} median {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
f.close()
