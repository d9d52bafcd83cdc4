"""K1 region clocks (diagnostic build with -DESLAM_K1_PROF): where a wave's time goes.

    python slam-eslam_amd/build_lib.py -DESLAM_K1_PROF
    ESLAM_GPU_LIB=slam-eslam_amd/lib/libeslam_gpu_eslam_k1_prof.so python tools/k1_prof.py
"""
import ctypes as C
import os
import sys

sys.path.insert(0, "slam-eslam_amd")
sys.path.insert(0, "tests")
import eslam_abi as A  # noqa: E402
import eslam_amd  # noqa: E402
import synthetic as S  # noqa: E402

NAMES = ["prologue", "gather", "load+philox+BM", "predict", "sincos(w)", "world+lookups", "contact logic",
         "evaluateWeight", "kalman+sw+stats", "stores+bbox", "chunk flush", "epilogue"]
n = int(os.environ.get("N", 4 * 1024 * 1024))
grid = S.flat_map(cells=1000)
stream = S.step_stream(40)
cfg = S.bench_config(A.default_config(), n)
f = eslam_amd.GpuFilter(cfg)
f.set_map(grid)
f.init_gaussian(n, [0, 0, 0], [0.1, 0.1, 0.1], 0.18, 1.001)
lib = eslam_amd.load_library()
fn = lib.eslam_debug_k1_prof
fn.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * 32)()
for st in stream[:5]:
    f.step(st)
f.sync()
fn(buf)
steps = 20
for st in stream[5:5 + steps]:
    f.step(st)
f.sync()
fn(buf)
marks = [0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12]
tot = sum(buf[k] for k in marks)
for name, k in zip(NAMES, marks):
    print(f"{name:18s} {buf[k] / tot * 100:6.1f} %   {buf[k] / steps / (n / 64):9.0f} clk/row")
print(f"total {tot / steps / (n / 64):.0f} clk per wave-row")
print(f"ratio path: {buf[14] / steps:.0f} waves/step, {buf[15] / steps:.0f} lane-contacts/step of {n * 4} "
      f"(rows {n / 64:.0f})")
K3 = ["load+normalize", "blocked fx", "scan+publish", "wait preds", "seek", "segments", "-", "flush marks"]
tot3 = sum(buf[16 + k] for k in range(len(K3)))
items = 2 if n <= 512 * 1024 else (4 if n <= 2 * 1024 * 1024 else 8)     # scan_items() of eslam_ctx.hip
waves3 = n / (64 * items)
for k, name in enumerate(K3):
    print(f"K3 {name:14s} {buf[16 + k] / max(tot3, 1) * 100:6.1f} %   {buf[16 + k] / steps / waves3:9.0f} clk/wave")
f.close()
