"""Localise a per-particle-map parity failure: GPU vs oracle after each stage of a few steps
(step, map update), field by field.  python tools/debug_maps.py [n] [steps] [empty]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "slam-eslam_amd"), os.path.join(ROOT, "tests")]
import eslam_abi as A  # noqa: E402
import eslam_amd  # noqa: E402
import oracle_ffi as O  # noqa: E402
import synthetic as S  # noqa: E402

FIELDS = ["x", "y", "orientation", "zpos", "zsigma", "weight", "mprob", "floating", "n_contact_points"]


def diff(tag, g, o):
    out = []
    for f in FIELDS:
        a, b = getattr(g, f), getattr(o, f)
        d = np.nonzero(np.any(np.ascontiguousarray(a).view(np.uint8).reshape(len(a), -1)
                              != np.ascontiguousarray(b).view(np.uint8).reshape(len(b), -1), axis=1))[0]
        if d.size:
            out.append(f"{f}:{d.size}(first {d[0]}: {a[d[0]]!r} vs {b[d[0]]!r})")
    print(tag, "OK" if not out else " ".join(out), flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    empty = len(sys.argv) > 3 and sys.argv[3] == "empty"
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    grid = S.unmapped_beyond(S.flat_map(cells=80), -1e9 if empty else 0.3)
    g = eslam_amd.GpuFilter(cfg)
    o = O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (g, o):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    scan = S.scan_patches()
    print("maps after init: gpu", len(g.particle_map(0)[0]), "oracle", len(o.particle_map(0)[0]))
    cfg2 = S.bench_config(A.default_config(), n)
    g2 = eslam_amd.GpuFilter(cfg2)
    g2.set_map(grid)
    g2.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    g2.step(S.step_stream(1)[0])
    print("gpu without maps: data particles", g2.sync().data_particles)
    for k, st in enumerate(S.step_stream(steps)):
        g.step(st)
        o.step(st)
        gi = g.sync()
        print("info gpu", gi.resampled, gi.data_particles, "oracle", o.info().resampled, o.info().data_particles)
        diff(f"step {k} after update:", g.download(), o.download())
        print("  anc equal:", np.array_equal(g.ancestors(), o.ancestors()))
        g.map_update(scan)
        o.map_update(scan)
        gi = g.sync()
        oi = o.info()
        print("  map info gpu", gi.map_patches_dropped, gi.map_stores_copied, gi.map_stores_changed, gi.map_patches_covered,
              "oracle", oi.map_patches_dropped, oi.map_stores_copied, oi.map_stores_changed, oi.map_patches_covered)
        diff(f"step {k} after map update:", g.download(), o.download())
        nbad = 0
        for i in range(n):
            gc, gm, gs = g.particle_map(i)
            oc, om, os_ = o.particle_map(i)
            gd = {int(c): (float(a), float(b)) for c, a, b in zip(gc, gm, gs)}
            od = {int(c): (float(a), float(b)) for c, a, b in zip(oc, om, os_)}
            if gd != od:
                nbad += 1
                if nbad <= 3:
                    only_g = sorted(set(gd) - set(od))[:6]
                    only_o = sorted(set(od) - set(gd))[:6]
                    vals = [(c, gd[c], od[c]) for c in sorted(set(gd) & set(od)) if gd[c] != od[c]][:4]
                    print(f"  map {i} differs: gpu {len(gd)} cells, oracle {len(od)}; only gpu {only_g} only oracle {only_o}"
                          f" values {vals}")
        print(f"  maps differing: {nbad} of {n}")


if __name__ == "__main__":
    main()
