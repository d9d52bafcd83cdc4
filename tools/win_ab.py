"""A/B: LDS map window on/off at small filter sizes (HIP events around 50 steps)."""
import sys, time
sys.path[:0] = ["slam-eslam_amd", "tests"]
import torch
import eslam_abi as A, eslam_amd, synthetic as S
grid = S.flat_map(cells=1000)
stream = S.step_stream(80)
for n in (65536, 262144, 1048576):
    for rep in range(2):
        for flag in (0, A.FLAG_NO_MAP_LDS):
            cfg = S.bench_config(A.default_config(), n)
            cfg.flags |= flag
            f = eslam_amd.GpuFilter(cfg)
            f.set_map(grid)
            f.init_gaussian(n, [0, 0, 0], [0.1, 0.1, 0.1], 0.18, 1.001)
            for st in stream[:10]: f.step(st)
            f.sync()
            t = time.perf_counter()
            for st in stream[10:60]: f.step(st)
            f.sync()
            dt = (time.perf_counter() - t) / 50
            print(n, "window" if not flag else "global", f"{dt*1e6:.1f} us/step", f"{n/dt/1e9:.2f} G/s", flush=True)
            del f
