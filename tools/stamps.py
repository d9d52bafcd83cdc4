"""Phase timeline of K1 and K3 from a -DESLAM_STAMPS diagnostic build (s_memrealtime, 10 ns):
    ESLAM_GPU_LIB=$PWD/slam-eslam_amd/lib/ab/lib_stamps.so python tools/stamps.py [particles] [warmup]
Runs the bench workload (flat map, resample forced) for `warmup` steps plus one, then prints,
per phase of the last step's K1 and K3 (the stamps are cleared before it, and the block
counts are the launches' own), the median / max block duration and when the last block left
the phase (from the kernel's first block start).  Read the shares, not the
lengths: the stamps' waits make the build slower than the product."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-eslam_amd"))

import eslam_abi as A  # noqa: E402
import eslam_amd  # noqa: E402
import synthetic as S  # noqa: E402

K1_PHASES = ["start", "window staged", "rows done", "stats flushed"]
K3_PHASES = ["start", "phase-B loads issued", "finalize seen", "phase B applied", "tile scanned",
             "look-back done", "draws counted", "marks written"]


def report(name, st, phases, nblocks):
    st = st[:nblocks, :len(phases)].astype(np.int64)
    done = np.all(st > 0, axis=1)                # blocks that returned early left zeros (cleared)
    st = st[done]
    if not len(st):
        print(f"== {name}: no block passed every phase")
        return
    t0 = st[:, 0].min()
    rel = (st - t0) * 10e-3                      # us
    print(f"== {name}: {nblocks} blocks ({len(st)} through every phase), span {rel[:, -1].max():.2f} us "
          "(first start to last end)")
    for k in range(1, len(phases)):
        d = rel[:, k] - rel[:, k - 1]
        print(f"  {phases[k - 1]:>22s} -> {phases[k]:<22s} median {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}"
              f"  max {d.max():7.2f} us; last block leaves at {rel[:, k].max():7.2f} us")
    starts = rel[:, 0]
    print(f"  block starts: median {np.median(starts):.2f}, p90 {np.percentile(starts, 90):.2f}, last {starts.max():.2f} us")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4 * 1024 * 1024
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    L = eslam_amd.load_library()
    L.eslam_gpu_debug_stamps.argtypes = [C.c_int, C.c_void_p, C.c_uint64]
    L.eslam_gpu_debug_stamps.restype = C.c_int64
    cfg = S.bench_config(A.default_config(), n)
    f = eslam_amd.GpuFilter(cfg, device=0)
    f.set_map(S.flat_map())
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    steps = list(S.step_stream(warm + 1))
    for st in steps[:-1]:
        f.step(st)
    f.sync()
    assert L.eslam_gpu_debug_stamps_clear() == 0  # the measured step's stamps only
    f.step(steps[-1])
    f.sync()
    buf = np.zeros((32768, 8), dtype=np.uint64)
    for which, label, phases in ((1, "K1", K1_PHASES), (3, "K3", K3_PHASES)):
        blocks = L.eslam_gpu_debug_stamps(which, buf.ctypes.data, 32768)
        assert blocks >= 0
        report(f"{label} at n={n} ({blocks} blocks launched)", buf.copy(), phases, min(blocks, 32768))
    f.close()


if __name__ == "__main__":
    main()
