"""Per-particle local maps on the CPU oracle (useSharedMap = false):
processMap's merge of a scan into every particle's map (src/EmbodiedSlamFilter.cpp:179-232)
and cloneMaps' private copies (src/PoseEstimator.cpp:31-47).  A particle's map is a window of
tiles of 8 x 8 cells reaching maxSensorRange around the particle, which moves
with it.  Pinned by the reference only in its insert-into-empty-cell rule
(test/testMap.cpp:307-316); envire's MLSGrid::merge is not in the reference, so the fuse rule
is the build's own (parity unpinned).  test_window_model restates the whole map update in
Python (exact rational arithmetic for the fused cell placement) as a second implementation."""
from fractions import Fraction
import math

import numpy as np
import pytest

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
        assert len(cells) == len(set(cells.tolist()))


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


def test_fuse_and_window(oracle):
    f, grid = setup(n=64, cells=120)
    scan = S.scan_patches()
    f.map_update(scan)
    assert f.info().map_patches_dropped == 0
    c1, m1, s1 = f.particle_map(5)
    f.map_update(scan)                                  # the same scan again: fused, variance halves
    c2, m2, s2 = f.particle_map(5)
    assert np.array_equal(c1, c2)
    assert np.all(s2 < s1) and np.all(np.abs(s2 - s1 / math.sqrt(2)) < 1e-5)
    # a scan reaching 5.5 m ahead: the patches beyond the window (4 tiles = 3.2-4.0 m from the
    # particle's tile at 0.1 m cells and maxSensorRange 3 m) are dropped and counted
    big = S.scan_patches(nx=12, ny=4, x0=0.35, x1=5.5, y0=-0.5, y1=0.5)
    f.map_update(big)
    assert f.info().map_patches_dropped > 0
    p = f.download()
    for i in (0, 5, 63):
        c3, _, _ = f.particle_map(i)
        c3 = c3.astype(np.int64)
        m, n = c3 % grid.width, c3 // grid.width
        pm = math.floor((p.x[i] - grid.offset[0]) / grid.scale[0]) >> 3
        pn = math.floor((p.y[i] - grid.offset[1]) / grid.scale[1]) >> 3
        assert np.all(np.abs((m >> 3) - pm) <= 4) and np.all(np.abs((n >> 3) - pn) <= 4)
        assert np.max(m) >= 8 * pm + 24                  # it reaches 3 tiles ahead


def test_window_forgets_what_it_leaves(oracle):
    """The robot walks 6 m: the tiles its window leaves are forgotten, nothing within
    maxSensorRange of the particle is dropped, and the map never holds more than the window."""
    n = 32
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    grid = S.unmapped_beyond(S.flat_map(cells=200), -1e9)          # the reference's empty start
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    scan = S.scan_patches()
    first = None
    for k, st in enumerate(S.step_stream(300, dx=0.02, dyaw=0.0)):
        f.step(st)
        f.map_update(scan)
        assert f.info().map_patches_dropped == 0, k
        if k == 10:
            first = set(f.particle_map(0)[0].tolist())
    last = set(f.particle_map(0)[0].tolist())
    assert first and not (first & last)                 # 6 m later the first cells are gone
    p = f.download()
    c, _, _ = f.particle_map(0)
    x = grid.offset[0] + (c % grid.width + 0.5) * grid.scale[0]
    assert np.all(np.abs(x - p.x[0]) < 4.1)
    assert np.mean(p.n_contact_points == 4) > 0.8       # the feet stand on merged cells only


def _fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _model_update(maps, p, scan, grid, sincos):
    """processMap on the window model: maps[i] = (centre, {tile: {cell_in_tile: (mean, sd)}})."""
    h, w = 4, 9
    inv_x, inv_y = 1.0 / grid.scale[0], 1.0 / grid.scale[1]
    drop = 0
    for i in range(len(maps)):
        ctr, tiles = maps[i]
        bx, by = p.x[i] - grid.offset[0], p.y[i] - grid.offset[1]
        nc = (math.floor(bx * inv_x) >> 3, math.floor(by * inv_y) >> 3)
        if nc != ctr:
            tiles = {t: v for t, v in tiles.items() if abs(t[0] - nc[0]) <= h and abs(t[1] - nc[1]) <= h}
            ctr = nc
        tiles = {t: dict(v) for t, v in tiles.items()}
        sn, co = sincos(p.orientation[i])
        zvar = p.zsigma[i] * p.zsigma[i]
        for k in range(len(scan)):
            sx, sy, sz = scan[k].position
            m = math.floor(_fma(co, sx, _fma(-sn, sy, bx)) * inv_x)
            n_ = math.floor(_fma(sn, sx, _fma(co, sy, by)) * inv_y)
            if not (0 <= m < grid.width and 0 <= n_ < grid.height):
                continue
            t = (m >> 3, n_ >> 3)
            if abs(t[0] - ctr[0]) > h or abs(t[1] - ctr[1]) > h:
                drop += 1
                continue
            wz = sz + p.zpos[i]
            var = scan[k].stdev * scan[k].stdev + zvar
            cells = tiles.setdefault(t, {})
            j = (m & 7) + 8 * (n_ & 7)
            if j in cells:
                m1, s1 = float(cells[j][0]), float(cells[j][1])
                v1, d = s1 * s1, wz - m1
                if d * d <= 9.0 * (v1 + var):
                    cells[j] = (np.float32((m1 * var + wz * v1) / (v1 + var)), np.float32(math.sqrt((v1 * var) / (v1 + var))))
            else:
                cells[j] = (np.float32(wz), np.float32(math.sqrt(var)))
        maps[i] = (ctr, tiles)
    return drop


@pytest.mark.parametrize("nx,ny,steps", [(10, 5, 40), (13, 10, 16)])
def test_window_model(oracle, nx, ny, steps):
    """The oracle's map update against the Python window model, cell for cell, over the bench
    stream (with its resample copies) on the empty prior and with a scan wide enough to reach
    past the window; the 130-patch scan is merged in parts of 64 (eslam_gpu_map_update), the
    model takes it whole."""
    n = 12
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    grid = S.unmapped_beyond(S.flat_map(cells=160), -1e9)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.3, 0.3, 0.2], 0.18, 0.05)
    scan = S.scan_patches(nx=nx, ny=ny, x0=-0.5, x1=4.2, y0=-1.5, y1=1.0)
    sincos = lambda th: (O.dm(2, th), O.dm(3, th))
    maps = [(None, {}) for _ in range(n)]
    for k, st in enumerate(S.step_stream(steps, dx=0.05)):
        f.step(st)
        anc = f.ancestors().astype(np.int64) if f.info().resampled else np.arange(n)
        maps = [maps[a] for a in anc]
        p = f.download()
        drop = _model_update(maps, p, scan, grid, sincos)
        f.map_update(scan)
        assert f.info().map_patches_dropped == drop, k
        for i in range(n):
            c, m, s_ = f.particle_map(i)
            want = {}
            for (ta, tb), cells in maps[i][1].items():
                for j, v in cells.items():
                    want[(8 * tb + j // 8) * grid.width + 8 * ta + j % 8] = v
            got = {int(cc): (mm, ss) for cc, mm, ss in zip(c, m, s_)}
            assert set(got) == set(want), (k, i)
            for cc, v in want.items():
                assert got[cc][0].view(np.uint32) == v[0].view(np.uint32) and got[cc][1].view(np.uint32) == v[1].view(np.uint32), (k, i, cc)


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


def flat_scan(dz=0.0, **kw):
    scan = S.scan_patches(**kw)
    for k in range(len(scan)):
        scan[k].position[2] = -0.18 + dz
    return scan


@pytest.mark.parametrize("rotated", [False, True])
def test_match_weights_against_own_map(oracle, rotated):
    """processMap(scanMap, match = true) (src/EmbodiedSlamFilter.cpp:214-221; the match rule is
    the build's own, envire's MLSGrid::match not being in the reference -- parity unpinned):
    against maps holding a flat scan, the same scan scores 1 on every cell (weights unchanged,
    bit for bit), a scan dz higher multiplies each matched particle's weight by
    float(exp(-dz^2 / (2 * 0.2f^2)))^0.1f and leaves the unmatched ones as they are, and only
    every 10th patch counts (sampling 10).  rotated: a grid whose global2local is a rotation and
    a shift (every cell placed through the transform)."""
    if rotated:
        cfg = S.bench_config(A.default_config(), 600)
        cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
        grid = S.unmapped_beyond(S.flat_map(cells=60), 0.3)
        c, s = math.cos(0.3), math.sin(0.3)
        grid.g2l = [c, s, 0.0, -(c * 0.4 + s * -0.25), -s, c, 0.0, -(-s * 0.4 + c * -0.25), 0.0, 0.0, 1.0, 0.0]
        f = O.OracleFilter(cfg, O.SUM_CONTRACT)
        f.set_map(grid)
        f.init_gaussian(600, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    else:
        f, _ = setup()
    f.step(S.step_stream(1)[0])                          # the weights of an update (init leaves 0)
    w_empty = f.download().weight.copy()
    assert np.all(w_empty > 0)
    f.map_match(flat_scan(0.1))                          # empty maps: nothing to match
    assert np.array_equal(f.download().weight, w_empty)
    scan = flat_scan()
    f.map_update(scan)
    w0 = f.download().weight.copy()
    f.map_match(scan)
    assert np.array_equal(f.download().weight, w0)
    odd = flat_scan()
    for k in range(len(odd)):
        if k % 10:
            odd[k].position[2] += 5.0                    # never sampled
    f.map_match(odd)
    assert np.array_equal(f.download().weight, w0)
    dz = 0.1
    f.map_match(flat_scan(dz))
    r = f.download().weight / w0
    sig = float(np.float32(0.2))
    score = float(np.float32(math.exp(-dz * dz / (2.0 * sig * sig))))
    expect = score ** float(np.float32(0.1))
    matched = np.abs(r - expect) < 1e-6
    assert np.all(matched | (r == 1.0))
    assert matched.mean() > 0.9
