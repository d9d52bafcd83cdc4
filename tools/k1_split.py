"""K1 time split on the GPU: project-only, update-only and full steps (HIP events)."""
import sys
import time

sys.path.insert(0, "slam-eslam_amd")
sys.path.insert(0, "tests")
import eslam_abi as A  # noqa: E402
import eslam_amd  # noqa: E402
import synthetic as S  # noqa: E402

n = 4 * 1024 * 1024
grid = S.flat_map(cells=1000)
stream = S.step_stream(200)


def run(flags, mode, steps=30):
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags = flags
    f = eslam_amd.GpuFilter(cfg)
    f.set_map(grid)
    f.init_gaussian(n, [0, 0, 0], [0.1, 0.1, 0.1], 0.18, 1.001)
    for st in stream[:5]:
        f.step(st)
    f.sync()
    f.enable_timing(True)
    t0 = time.perf_counter()
    for st in stream[5:5 + steps]:
        if mode == "project":
            f.project(st)
        elif mode == "update":
            f.update(st)
        else:
            f.step(st)
    f.sync()
    dt = (time.perf_counter() - t0) / steps
    kt = f.kernel_times()
    f.close()
    return dt * 1e3, kt["project_weight_ms"]


modes = sys.argv[1:] or ["project", "update", "step"]
configs = ((0, "lds-window"), (A.FLAG_NO_MAP_LDS, "global-map")) if len(sys.argv) == 1 else ((0, "lds-window"),)
for flags, name in configs:
    for mode in modes:
        ms, k1 = run(flags, mode)
        print(f"{name:11s} {mode:8s} step {ms:.4f} ms  K1 {k1 * 1e3:.1f} us", flush=True)
