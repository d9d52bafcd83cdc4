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


def test_insert_into_empty_cells(oracle):
    f, grid = setup()
    scan = S.scan_patches(x0=0.45)                       # clear of the mapped cells x < 0.3
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


def loop_walk(trail, n=32, out=300, back=260):
    """6 m out and (nearly) back on the empty prior with a map update after every step; returns
    the filter, the first cells particle 0 mapped, the found-contact fraction per step of the
    way back and the evictions"""
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    cfg.local_map_trail = trail
    grid = S.unmapped_beyond(S.flat_map(cells=200), -1e9)          # the reference's empty start
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    scan = S.scan_patches()
    first, found_back, evicted = None, [], 0
    stream = S.step_stream(out, dx=0.02, dyaw=0.0) + S.step_stream(back, dx=-0.02, dyaw=0.0)
    for k, st in enumerate(stream):
        f.step(st)
        f.map_update(scan)
        assert f.info().map_patches_dropped == 0, k
        evicted += f.info().map_tiles_evicted
        if k == 10:
            first = set(f.particle_map(0)[0].tolist())
        if k >= out:
            found_back.append(float(np.mean(f.download().n_contact_points == 4)))
    return f, grid, first, found_back, evicted


def test_trail_keeps_what_the_window_leaves(oracle):
    """The robot walks 6 m and back (the reference keeps every grid its MLSMap made,
    src/EmbodiedSlamFilter.cpp:195-207): the tiles the window leaves go to the trail, and on the
    way back the feet find the cells mapped on the way out -- the scan looks ahead in +x, so
    walking back it never maps the cells under the feet itself.  Without a trail they are
    forgotten and the feet find nothing.  A trail larger than the walk needs changes no bit."""
    f, grid, first, found, ev = loop_walk(16)
    g, _, first0, found0, ev0 = loop_walk(0)
    h, _, _, found_big, ev_big = loop_walk(64)
    assert ev == 0 and ev_big == 0 and ev0 > 0
    # the last 80 steps (1.6 m) of the way back: more than 3.2 m from where the walk turned
    assert np.mean(found[-80:]) > 0.9 and min(found[-80:]) > 0.7, found   # the cells of the way out
    assert max(found0[-80:]) < 0.05, found0             # forgotten without a trail
    last = set(f.particle_map(0)[0].tolist())
    assert first <= last                                # the first cells are still held
    assert first0 and not (first0 & set(g.particle_map(0)[0].tolist()))
    pf, ph = f.download(), h.download()
    for fld in ("x", "y", "orientation", "zpos", "zsigma", "weight"):
        assert np.array_equal(getattr(pf, fld), getattr(ph, fld)), fld
    for i in (0, 7, 31):
        c1, m1, s1 = f.particle_map(i)
        c2, m2, s2 = h.particle_map(i)
        assert sorted(zip(c1.tolist(), m1.tolist(), s1.tolist())) == sorted(zip(c2.tolist(), m2.tolist(), s2.tolist()))


def _fma(a, b, c):
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _model_recentre(ctr, tiles, trail, nc, h, w):
    """the window moves from ctr to nc: the tiles leaving it go to the trail in slot order -- an
    empty entry, else in place of the entry farthest from nc (Chebyshev, the first of them) if
    that is farther than the tile -- then the trail's tiles inside the new window come back;
    returns the new (tiles, trail) and the tiles forgotten"""
    inside = lambda t: abs(t[0] - nc[0]) <= h and abs(t[1] - nc[1]) <= h
    dist = lambda t: max(abs(t[0] - nc[0]), abs(t[1] - nc[1]))
    keep = {t: v for t, v in tiles.items() if inside(t)}
    leaving = sorted((t for t in tiles if not inside(t)), key=lambda t: (t[0] % w) + w * (t[1] % w))
    trail = list(trail)
    forgot = 0
    for t in leaving:
        if None in trail:
            trail[trail.index(None)] = (t, tiles[t])
            continue
        forgot += 1
        if trail:
            far = max(range(len(trail)), key=lambda e: (dist(trail[e][0]), -e))
            if dist(trail[far][0]) > dist(t):
                trail[far] = (t, tiles[t])
    for e, ent in enumerate(trail):
        if ent is not None and inside(ent[0]):
            keep[ent[0]] = ent[1]
            trail[e] = None
    return keep, trail, forgot


def _model_update(maps, p, scan, grid, sincos):
    """processMap on the window model: maps[i] = (centre, {tile: {cell_in_tile: (mean, sd)}},
    trail [(tile, cells) or None] * V)."""
    h, w = 4, 9
    inv_x, inv_y = 1.0 / grid.scale[0], 1.0 / grid.scale[1]
    drop = forgot = 0
    for i in range(len(maps)):
        ctr, tiles, trail = maps[i]
        bx, by = p.x[i] - grid.offset[0], p.y[i] - grid.offset[1]
        nc = (math.floor(bx * inv_x) >> 3, math.floor(by * inv_y) >> 3)
        if nc != ctr:
            if ctr is not None:
                tiles, trail, fg = _model_recentre(ctr, tiles, trail, nc, h, w)
                forgot += fg
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
        maps[i] = (ctr, tiles, trail)
    return drop, forgot


@pytest.mark.parametrize("nx,ny,steps,dx,trail", [(10, 5, 40, 0.05, 16), (13, 10, 16, 0.05, 16), (10, 5, 40, 0.15, 16),
                                                 (10, 5, 40, 0.15, 3), (10, 5, 30, 0.15, 0)])
def test_window_model(oracle, nx, ny, steps, dx, trail):
    """The oracle's map update against the Python window model, cell for cell, over the bench
    stream (with its resample copies) on the empty prior and with a scan wide enough to reach
    past the window; the 130-patch scan is merged in parts of 64 (eslam_gpu_map_update), the
    model takes it whole.  dx 0.15: the windows move 6 m, tiles go to the trail (3 entries: it
    overflows and forgets the farthest; 0: no trail)."""
    n = 12
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    cfg.local_map_trail = trail
    grid = S.unmapped_beyond(S.flat_map(cells=240), -1e9)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.3, 0.3, 0.2], 0.18, 0.05)
    scan = S.scan_patches(nx=nx, ny=ny, x0=-0.5, x1=4.2, y0=-1.5, y1=1.0)
    sincos = lambda th: (O.dm(2, th), O.dm(3, th))
    maps = [(None, {}, [None] * trail) for _ in range(n)]
    evicted = 0
    for k, st in enumerate(S.step_stream(steps, dx=dx)):
        f.step(st)
        anc = f.ancestors().astype(np.int64) if f.info().resampled else np.arange(n)
        maps = [maps[a] for a in anc]
        p = f.download()
        drop, forgot = _model_update(maps, p, scan, grid, sincos)
        f.map_update(scan)
        assert f.info().map_patches_dropped == drop, k
        assert f.info().map_tiles_evicted == forgot, k
        evicted += forgot
        for i in range(n):
            c, m, s_ = f.particle_map(i)
            want = {}
            held = list(maps[i][1].items()) + [e for e in maps[i][2] if e is not None]
            for (ta, tb), cells in held:
                for j, v in cells.items():
                    want[(8 * tb + j // 8) * grid.width + 8 * ta + j % 8] = v
            got = {int(cc): (mm, ss) for cc, mm, ss in zip(c, m, s_)}
            assert set(got) == set(want), (k, i)
            for cc, v in want.items():
                assert got[cc][0].view(np.uint32) == v[0].view(np.uint32) and got[cc][1].view(np.uint32) == v[1].view(np.uint32), (k, i, cc)
    if dx > 0.1:
        assert (evicted > 0) == (trail < 16), evicted


def test_scan_on_mapped_cells_fuses_with_the_grid(oracle):
    """A scan patch on a cell the shared grid covers goes into the particle's own copy of the
    cell (the reference merges into each particle's clone of the grid, src/EmbodiedSlamFilter.cpp:
    222-227, clones at src/PoseEstimator.cpp:31-62): fused with the grid's patch (flat map: mean
    0, stdev 0.05) when within 3 sigma; the contact update then reads the particle's patch."""
    f, grid = setup(n=200)
    back = S.scan_patches(nx=8, ny=6, x0=-0.6, x1=0.95)
    f.map_update(back)
    p = f.download()
    cs = grid.cell_start.astype(np.int64)
    g_sd = float(np.float32(0.05))
    seen = 0
    for i in range(0, p.n, 13):
        cells, mean, sd = f.particle_map(i)
        cov = cs[cells.astype(np.int64)] != cs[cells.astype(np.int64) + 1]
        seen += int(cov.sum())
        zs2 = p.zsigma[i] * p.zsigma[i]
        var = 0.03 * 0.03 + zs2
        v1 = g_sd * g_sd
        want_sd = np.float32(math.sqrt((v1 * var) / (v1 + var)))
        # fused with the grid's patch at least once: at most the fusion of one grid and one scan
        # patch (a cell two scan patches reach fuses twice)
        assert np.all(sd[cov] <= want_sd + 2e-7), (i, sd[cov], want_sd)
        assert np.any(np.abs(sd[cov] - want_sd) < 2e-7) or not cov.any()
    assert seen > 0


def test_covered_cells_are_counted(oracle):
    """Scan patches on cells the shared grid covers go into the particle's copy of the cell
    (test_scan_on_mapped_cells_fuses_with_the_grid) and are counted (map_patches_covered): a scan reaching back over the mapped region x < 0.3."""
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
    kw.setdefault("x0", 1.2)                # far enough ahead that no patch lands on the mapped
    kw.setdefault("x1", 1.8)                # cells x < 0.3 (rotated grid included)
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
    a shift (every cell placed through the transform).  The scan lies on cells the shared grid
    leaves empty (its own cells: test_match_against_the_shared_grid)."""
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


def match_expect(p, dz, sd_scan=0.03, grid_sd=0.05):
    """closed form of the shared-grid rule on the flat map (mean 0): every sampled patch of a
    particle lands on a grid cell at local height -0.18 + dz + zPos, so its score is the same
    for all of them: exp(-d^2 / (2 * 0.2f^2)) when the 3-sigma gate passes, else 0"""
    sig = float(np.float32(0.2))
    d = -0.18 + dz + p.zpos
    qv = sd_scan * sd_scan + p.zsigma * p.zsigma
    gs = float(np.float32(grid_sd))
    score = np.where(d * d < 9.0 * (gs * gs + qv), np.exp(-(d * d) / (2.0 * sig * sig)), 0.0)
    wf = score.astype(np.float32).astype(np.float64)
    return wf ** float(np.float32(0.1))


@pytest.mark.parametrize("pmaps", [False, True])
def test_match_against_the_shared_grid(oracle, pmaps):
    """processMap(scanMap, match = true) with the shared map (useSharedMap = true: the laser
    path's match-only call, src/EmbodiedSlamFilter.cpp:214-221,342-344), and the grid's cells of
    a per-particle map (the clone the reference merges into holds them): each sampled patch
    scores against the patch getPatch's 3-sigma gate picks in its cell (0 when none passes);
    patches off the grid do not count (weights unchanged)."""
    n = 400
    cfg = S.bench_config(A.default_config(), n)
    if pmaps:
        cfg.flags |= A.FLAG_PARTICLE_MAPS
    grid = S.flat_map(cells=60)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(grid)
    f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    f.step(S.step_stream(1)[0])
    for dz in (0.0, 0.07, 0.5):
        p = f.download()
        w0 = p.weight.copy()
        f.map_match(flat_scan(dz, x0=0.35, x1=0.95))
        r = f.download().weight / w0
        want = match_expect(p, dz)
        assert np.allclose(r, want, rtol=1e-12, atol=0.0), (dz, np.max(np.abs(r - want)))
        if dz == 0.5:
            assert np.all(r == 0.0)                      # no patch within 3 sigma: score 0
        else:
            f.upload(p)                                  # back to the weights before the match
    f2 = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f2.set_map(grid)
    f2.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    f2.step(S.step_stream(1)[0])
    w0 = f2.download().weight.copy()
    f2.map_match(flat_scan(0.0, x0=40.0, x1=41.0))        # beyond the 6 m grid: nothing counts
    assert np.array_equal(f2.download().weight, w0)
