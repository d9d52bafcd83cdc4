"""Per-particle local maps on the CPU oracle (useSharedMap = false):
processMap's merge of a scan into every particle's map (src/EmbodiedSlamFilter.cpp:179-232)
and cloneMaps' private copies (src/PoseEstimator.cpp:31-47).  Pinned by the reference only in
its insert-into-empty-cell rule (test/testMap.cpp:307-316); envire's MLSGrid::merge is not in
the reference, so the fuse rule is the build's own (parity unpinned)."""
import math

import numpy as np

import eslam_abi as A
import oracle_ffi as O
import synthetic as S


def setup(n=600, x0=0.3, cells=60):
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    grid = S.unmapped_beyond(S.flat_map(cells=cells), x0)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    return f, grid


def test_insert_into_empty_cells_only(oracle):
    f, grid = setup()
    scan = S.scan_patches()
    f.map_update(scan)
    p = f.download()
    cs = grid.cell_start
    for i in range(0, p.n, 37):
        cells, mean, sd = f.particle_map(i)
        assert len(cells) > 0
        assert np.all(cs[cells] == cs[cells + 1]), "a shared-grid cell was written"
        # each patch is a scan patch placed at the particle: mean = z + zPos, sd = sqrt(s^2 + zs^2)
        # (two scan patches in one cell fuse: sd / sqrt(2))
        s0 = math.sqrt(0.03 ** 2 + p.zsigma[i] ** 2)
        assert np.all((np.abs(sd - s0) < 1e-6) | (np.abs(sd - s0 / math.sqrt(2)) < 1e-6))
        assert np.all(np.abs(mean - (p.zpos[i] - 0.18)) < 0.011)
        assert len(cells) == len(set(cells.tolist())) <= 24


def test_maps_follow_the_particles_and_answer_lookups(oracle):
    """The feet walk into the unmapped region: with the scans merged ahead of them the
    particles keep finding contact points there; the resample deep-copies the maps."""
    f, grid = setup()
    g, _ = setup()                                      # the same filter without map updates
    scan = S.scan_patches()
    found, found_without = [], []
    for k, st in enumerate(S.step_stream(30)):
        f.step(st)
        f.map_update(scan)
        g.step(st)
        p = f.download()
        found.append(float(np.mean(p.n_contact_points == 4)))
        found_without.append(float(np.mean(g.download().n_contact_points == 4)))
        anc = f.ancestors()
        if k == 20:
            # outputs of one ancestor hold equal maps after the (deep-copying) resample
            a = anc.astype(np.int64)
            i = int(np.argmax(np.diff(a) == 0))
            c1, m1, s1 = f.particle_map(i)
            c2, m2, s2 = f.particle_map(i + 1)
            assert np.array_equal(np.sort(c1), np.sort(c2))
    # by step 20 the front feet are at x > 0.55: beyond x0 = 0.3, found only in the local maps
    assert min(found[20:]) > 0.8, found
    assert max(found_without[20:]) < 0.05, found_without


def test_fuse_and_capacity(oracle):
    f, grid = setup(n=64)
    scan = S.scan_patches()
    f.map_update(scan)
    c1, m1, s1 = f.particle_map(5)
    f.map_update(scan)                                  # the same scan again: fused, variance halves
    c2, m2, s2 = f.particle_map(5)
    assert np.array_equal(c1, c2)
    assert np.all(s2 < s1) and np.all(np.abs(s2 - s1 / math.sqrt(2)) < 1e-5)
    big = S.scan_patches(nx=8, ny=8, x0=0.35, x1=3.0, y0=-2.0, y1=2.0)
    f.map_update(big)
    c3, _, _ = f.particle_map(5)
    assert len(c3) == 24                                # at most 24 patches per particle


def test_covered_cells_are_counted(oracle):
    """Scan patches on cells the shared grid covers are not merged and are
    counted (map_patches_covered): a scan reaching back over the mapped region x < 0.3."""
    f, grid = setup(n=200)
    back = S.scan_patches(nx=8, ny=6, x0=-0.6, x1=0.95)
    f.map_update(back)
    info = f.info()
    p = f.download()
    # recount on the host: every placed scan patch of every particle on a covered cell
    cs = grid.cell_start.astype(np.int64)
    covered = 0
    for i in range(p.n):
        c, s = math.cos(p.orientation[i]), math.sin(p.orientation[i])
        for k in range(len(back)):
            sx, sy = back[k].position[0], back[k].position[1]
            m = math.floor((c * sx - s * sy + p.x[i] - grid.offset[0]) / grid.scale[0])
            n_ = math.floor((s * sx + c * sy + p.y[i] - grid.offset[1]) / grid.scale[1])
            if 0 <= m < grid.width and 0 <= n_ < grid.height:
                cell = n_ * grid.width + m
                covered += int(cs[cell + 1] != cs[cell])
    assert info.map_patches_covered > 0
    # the host recount uses plain double arithmetic: it may differ from the contract's cell
    # placement (fma, 1/scale) on a handful of boundary patches
    assert abs(int(info.map_patches_covered) - covered) <= max(3, covered // 500)
