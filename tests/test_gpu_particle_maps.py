"""Per-particle local maps on the GPU (useSharedMap = false): every
particle's map is the shared grid plus its own window of tiles reaching maxSensorRange
(eslam_gpu_map_update = processMap's merge, src/EmbodiedSlamFilter.cpp:179-232; DESIGN.md
5c), copied on write after a resample (cloneMaps, src/PoseEstimator.cpp:31-47), read by the
contact update.  Bit-exact against the oracle, which copies every map at every resample:
particles after every step and every particle's own patches.  The empty prior is the
reference's own start with useSharedMap = false (every particle clones an empty grid
template, src/EmbodiedSlamFilter.cpp:131-134).  Parity with the reference is pinned only by
the insert-into-empty-cell rule (test/testMap.cpp:307-316); the fuse rule is the build's own."""
import numpy as np
import pytest

import eslam_abi as A
import oracle_ffi as O
import synthetic as S
from parity_util import assert_bit_identical

pytestmark = pytest.mark.gpu


def u32(a):
    return np.ascontiguousarray(a).view(np.uint32)


MAP_INFO = ("map_patches_dropped", "map_stores_copied", "map_stores_changed", "map_patches_covered", "map_tiles_evicted")


def map_info(i):
    return tuple(int(getattr(i, f)) for f in MAP_INFO)


def assert_maps_equal(gpu, orc, idx, label):
    for i in idx:
        gc, gm, gs = gpu.particle_map(i)
        oc, om, os_ = orc.particle_map(i)
        go, oo = np.argsort(gc), np.argsort(oc)
        assert np.array_equal(gc[go], oc[oo]), (label, i)
        assert np.array_equal(u32(gm[go]), u32(om[oo])) and np.array_equal(u32(gs[go]), u32(os_[oo])), (label, i)


@pytest.mark.parametrize("terrain,n,records", [("flat", 600, False), ("rough", 5003, False), ("rough", 2048, True)])
def test_particle_maps_bit_exact(gpu_mod, oracle, terrain, n, records):
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    if records:
        cfg.flags |= A.FLAG_RECORD_CONTACTS
    base = S.flat_map(cells=80) if terrain == "flat" else S.rough_map(cells=80)
    grid = S.unmapped_beyond(base, 0.3)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    if records:
        orc.set_debug(True)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    scan = S.scan_patches()
    stream = S.step_stream(24, tilt=(terrain == "rough"))
    dropped = 0
    for k, st in enumerate(stream):
        assert gpu.step(st) == orc.step(st)
        gpu.map_update(scan)
        orc.map_update(scan)
        gi = gpu.sync()
        assert_bit_identical(gpu.download(), orc.download(), f"{terrain} n={n} step {k}")
        # a full store's dropped patches, the copy-on-write copies and the changed stores
        # of every map update equal the oracle's (deep copies, open-addressing stores)
        assert map_info(gi) == map_info(orc.info()), (k, map_info(gi), map_info(orc.info()))
        dropped += gi.map_patches_dropped
        if k % 6 == 5:
            for i in list(range(0, n, max(n // 40, 1))) + [n - 1]:
                gc, gm, gs = gpu.particle_map(i)
                oc, om, os_ = orc.particle_map(i)
                go, oo = np.argsort(gc), np.argsort(oc)
                assert np.array_equal(gc[go], oc[oo]), (k, i)
                assert np.array_equal(u32(gm[go]), u32(om[oo])) and np.array_equal(u32(gs[go]), u32(os_[oo])), (k, i)
    assert dropped == 0                  # every scan patch lies within maxSensorRange
    if records:
        rec, cps = gpu.download_records(max_cpoints=4)
        ncp, cp, _, _ = orc.debug()
        anc = orc.ancestors().astype(np.int64)
        assert np.array_equal(rec["n_cpoints"], ncp[anc])
    # the front feet stand beyond x0 = 0.3 on cells only the scans mapped (on the rough map
    # the rear feet's terrain and the flat scan disagree more often)
    p = gpu.download()
    assert np.mean(p.n_contact_points == 4) > (0.5 if terrain == "flat" else 0.1)


def prior(kind, cells):
    base = S.rough_map(cells=cells)
    return S.unmapped_beyond(base, 0.3 if kind == "current" else -1e9)


@pytest.mark.parametrize("kind", ["current", "empty"])
def test_particle_maps_steady_state(gpu_mod, oracle, kind):
    """The bench workload run into the steady state: 45 steps move the robot 0.9 m (the window
    moves and forgets tiles), with the call patterns around the merge's fused resample gather: a
    step with no map update before the next step (the step gathers), two map updates in a row
    (the second finds no gather pending), and no download in between.  Bit-exact against the
    oracle: every step's map-update counts, then every particle and sampled maps.  In the steady
    state no scan patch is dropped and the feet find the merged cells."""
    n = 65536
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    grid = prior(kind, 300)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_threads(16)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    scan = S.scan_patches()
    for k, st in enumerate(S.step_stream(45, tilt=True)):
        assert gpu.step(st) == orc.step(st)
        if k % 10 == 7:
            continue                      # no map update: the next step runs the gather
        reps = 2 if k % 10 == 3 else 1    # a second update finds no gather pending
        for _ in range(reps):
            gpu.map_update(scan)
            orc.map_update(scan)
            assert map_info(gpu.sync()) == map_info(orc.info()), k
    info = gpu.sync()
    assert_bit_identical(gpu.download(), orc.download(), f"local maps steady state ({kind} prior)")
    assert np.array_equal(gpu.ancestors(), orc.ancestors())
    assert_maps_equal(gpu, orc, [0, 1, 977, n // 3, n // 2 + 5, n - 1], "steady state")
    assert info.map_patches_dropped == 0 and info.map_stores_changed == n
    assert info.data_particles > 0.8 * n                     # the feet stand on merged cells


def test_particle_maps_page_collection(gpu_mod, oracle):
    """A page pool of 10 pages per particle (the steady state names about 5): the collection (mark the pages live tables name,
    compact the rest) runs every few map updates; 60 steps stay bit-exact against the oracle,
    which has no pool.  Then 1 page per particle: the pool cannot hold a map update, the update
    writes nothing and the filter reports ESLAM_ERR_OUT_OF_MEMORY until it is re-initialised."""
    n = 8192
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    cfg.local_map_pages = 10
    grid = prior("empty", 200)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_threads(16)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    scan = S.scan_patches()
    for k, st in enumerate(S.step_stream(60, tilt=True)):
        assert gpu.step(st) == orc.step(st)
        gpu.map_update(scan)
        orc.map_update(scan)
        assert map_info(gpu.sync()) == map_info(orc.info()), k
    assert_bit_identical(gpu.download(), orc.download(), "page collection")
    assert_maps_equal(gpu, orc, [0, 5, n // 2, n - 1], "page collection")
    gpu.close()
    cfg.local_map_pages = 1
    g2 = gpu_mod.GpuFilter(cfg)
    g2.set_map(grid)
    g2.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    stream = S.step_stream(6, tilt=True)
    with pytest.raises(gpu_mod.EslamError) as ei:
        for st in stream:
            g2.step(st)
            g2.map_update(scan)
            g2.sync()
    assert ei.value.code == A.ERR_OUT_OF_MEMORY
    g2.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)   # starts over
    g2.step(stream[0])
    g2.sync()


def test_set_map_clears_particle_maps(gpu_mod):
    n = 1000
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    gpu = gpu_mod.GpuFilter(cfg)
    grid = prior("empty", 100)
    gpu.set_map(grid)
    gpu.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    gpu.step(S.step_stream(1)[0])
    gpu.map_update(S.scan_patches())
    assert len(gpu.particle_map(3)[0]) > 0
    gpu.set_map(grid)
    assert len(gpu.particle_map(3)[0]) == 0


def test_map_update_needs_the_flag(gpu_mod):
    cfg = S.bench_config(A.default_config(), 100)
    gpu = gpu_mod.GpuFilter(cfg)
    gpu.set_map(S.flat_map(cells=50))
    gpu.init_gaussian(100, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    with pytest.raises(gpu_mod.EslamError):
        gpu.map_update(S.scan_patches())


@pytest.mark.parametrize("kind,match", [("current", False), ("empty", False), ("current", True)])
def test_particle_maps_bench_workload(gpu_mod, oracle, kind, match):
    """bench.py --local-maps' workload (configs[4]'s terrain: rough multi-patch map, unmapped
    beyond x = 0.3 m -- or the reference's empty start --, tilted body, one map update per
    step; with match, `--local-maps --match`: the match weighting before every merge) at 256k
    particles on the 1000 x 1000 map: bit-exact against the oracle (16 threads) for 4 steps,
    and the maps of sampled particles equal."""
    n = 262144
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    grid = prior(kind, 1000)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_threads(16)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    scan = S.scan_patches()
    for k, st in enumerate(S.step_stream(4, tilt=True)):
        assert gpu.step(st) == orc.step(st)
        if match:
            gpu.map_match(scan)
            orc.map_match(scan)
        gpu.map_update(scan)
        orc.map_update(scan)
        assert map_info(gpu.sync()) == map_info(orc.info()), k
    assert_bit_identical(gpu.download(), orc.download(), f"local maps 256k ({kind} prior, match {match})")
    assert_maps_equal(gpu, orc, [0, 1, 4097, n // 2, n - 1], "256k")
    if kind == "current":
        assert np.mean(gpu.download().n_contact_points >= 2) > 0.1


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("kind", ["current", "empty"])
def test_particle_maps_config4_shard_size(gpu_mod, oracle, kind):
    """configs[4] at its per-GPU size: 8M particles (64M over 8 GPUs) with per-particle
    maps on the bench workload, 3 steps, bit-exact against the oracle (16 threads): every
    particle after the last step, the map-update counts of every step, and the maps of 40
    sampled particles."""
    n = 8 * 1024 * 1024
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    grid = prior(kind, 1000)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_threads(16)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    scan = S.scan_patches()
    for k, st in enumerate(S.step_stream(3, tilt=True)):
        assert gpu.step(st) == orc.step(st)
        gpu.map_update(scan)
        orc.map_update(scan)
        assert map_info(gpu.sync()) == map_info(orc.info()), k
    assert_bit_identical(gpu.download(), orc.download(), f"local maps 8M ({kind} prior)")
    idx = sorted(set(np.linspace(0, n - 1, 38).astype(np.int64).tolist() + [1, n // 2 + 1]))
    assert_maps_equal(gpu, orc, idx, "8M")
    gpu.close()


def rotated(grid, yaw=0.3, tx=0.4, ty=-0.25):
    """the grid in a local frame rotated by yaw and shifted: global2local = Rz(-yaw) (p - t)"""
    import math
    c, s = math.cos(yaw), math.sin(yaw)
    grid.g2l = [c, s, 0.0, -(c * tx + s * ty), -s, c, 0.0, -(-s * tx + c * ty), 0.0, 0.0, 1.0, 0.0]
    return grid


@pytest.mark.parametrize("case", ["wide_scan", "rotated_grid", "small_window", "large_window", "laser_scan", "mapped_cells"])
def test_particle_maps_shapes(gpu_mod, oracle, case):
    """The window's other shapes against the oracle, bit for bit: a scan reaching more tiles than
    one merge pass holds (kLmList = 8: the plan's and the merge's later passes) and past the
    window (dropped patches); a grid whose global2local is not the identity (every cell placed
    through the transform, in the plan, the merge and K1's lookups); a 5 x 5-tile window
    (maxSensorRange 1 m) and a 27 x 27-tile one (10 m, reaching past the grid's edges); a laser
    scan's MLS of 600 patches at the map's resolution (parts of 256: the large plan and merge, and a
    last part of 88); a scan reaching back over the mapped cells (each particle's copy of a
    shared-grid cell starts from the grid's patch, and its lookups then ask its own cells first)."""
    n = 1500
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    grid = S.unmapped_beyond(S.rough_map(cells=120), 0.3)
    scan = S.scan_patches()
    if case == "wide_scan":
        scan = S.scan_patches(nx=16, ny=12, x0=-2.6, x1=4.6, y0=-2.5, y1=2.4)   # 192 patches: three parts of 64
        cfg.local_map_pages = 128            # ~50 tiles a particle and its copies' pages
    elif case == "rotated_grid":
        grid = rotated(grid)
    elif case == "mapped_cells":
        scan = S.scan_patches(nx=10, ny=6, x0=-0.9, x1=0.95)
        cfg.local_map_pages = 48
    elif case == "laser_scan":
        scan = S.scan_area(600)
        cfg.local_map_pages = 48             # ~16 tiles a particle and its copies' pages
    elif case == "small_window":
        cfg.max_sensor_range = 1.0
        scan = S.scan_patches(nx=10, ny=8, x0=-0.8, x1=1.9, y0=-1.2, y1=1.0)
        cfg.local_map_pages = 48             # the scan reaches back over the mapped cells: their copies
    else:
        cfg.max_sensor_range = 10.0
        scan = S.scan_patches(nx=12, ny=10, x0=-5.0, x1=5.5, y0=-4.0, y1=4.0)
        cfg.local_map_pages = 256            # up to 120 tiles a particle
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.05], 0.18, 0.05)
    dropped = written = 0
    for k, st in enumerate(S.step_stream(12, tilt=True)):
        assert gpu.step(st) == orc.step(st)
        gpu.map_update(scan)
        orc.map_update(scan)
        gi = gpu.sync()
        assert_bit_identical(gpu.download(), orc.download(), f"{case} step {k}")
        assert map_info(gi) == map_info(orc.info()), (case, k, map_info(gi), map_info(orc.info()))
        dropped += gi.map_patches_dropped
        written += gi.map_cells_written
    assert_maps_equal(gpu, orc, list(range(0, n, 97)) + [n - 1], case)
    assert written > 0
    if case in ("wide_scan", "small_window"):
        assert dropped > 0                   # the scan reaches past the window
    else:
        assert dropped == 0
    if case == "mapped_cells":
        assert gi.map_patches_covered > 0


@pytest.mark.parametrize("case", ["identity", "rotated_grid", "mapped_cells"])
def test_particle_maps_match_bit_exact(gpu_mod, oracle, case):
    """processMap(scanMap, match, update) (src/EmbodiedSlamFilter.cpp:179-232): the match
    weighting (eslam_gpu_map_match: every 10th patch scored against the particle's own map,
    w *= pow(weight, 0.1f); the rule is the build's own) before the merge, with
    match-only and update-only calls mixed in and the weights feeding the next step's resample;
    a match against empty maps first.  Bit-exact against the oracle after every call."""
    n = 5003
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    grid = S.unmapped_beyond(S.rough_map(cells=120), 0.3)
    if case == "rotated_grid":
        grid = rotated(grid)
    if case == "mapped_cells":
        cfg.local_map_pages = 48                      # copies of the mapped cells the scans reach
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.05], 0.18, 0.05)
    scan = S.scan_patches(nx=12, ny=9)                # 108 patches: 11 sampled
    probe = S.scan_patches(nx=12, ny=9, z=-0.15)
    if case == "mapped_cells":                        # reaching back over the shared grid's cells
        scan = S.scan_patches(nx=12, ny=9, x0=-0.9, x1=0.95)
        probe = S.scan_patches(nx=12, ny=9, x0=-0.9, x1=0.95, z=-0.15)
    lowered = 0
    for k, st in enumerate(S.step_stream(14, tilt=True)):
        assert gpu.step(st) == orc.step(st)
        w0 = gpu.download().weight.copy()
        if k % 4 != 2:                                # processMap(scan, true, ...)
            gpu.map_match(probe)
            orc.map_match(probe)
            assert_bit_identical(gpu.download(), orc.download(), f"{case} match step {k}")
            lowered += int(np.sum(gpu.download().weight < w0))
        if k % 4 != 1:                                # processMap(scan, ..., true)
            gpu.map_update(scan)
            orc.map_update(scan)
            assert map_info(gpu.sync()) == map_info(orc.info()), (case, k)
        assert_bit_identical(gpu.download(), orc.download(), f"{case} step {k}")
    assert np.array_equal(gpu.ancestors(), orc.ancestors())
    assert lowered > n                                # the probe scan sits 3 cm above the maps


def test_particle_maps_match_edges(gpu_mod, oracle):
    """eslam_gpu_map_match's edges: an empty scan (weight 1: weights unchanged, bit for bit), a
    scan of fewer than 10 patches (only patch 0 sampled), non-finite patches (ESLAM_ERR_INVALID_ARG,
    nothing changed) and a filter with the shared map only (the grid's cells: as the oracle)."""
    n = 700
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS
    grid = S.unmapped_beyond(S.flat_map(cells=80), 0.3)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    scan = S.scan_patches()
    for st in S.step_stream(3):
        assert gpu.step(st) == orc.step(st)
        gpu.map_update(scan)
        orc.map_update(scan)
    w0 = gpu.download().weight.copy()
    empty = (A.ScanPatch * 0)()
    gpu.map_match(empty)
    orc.map_match(empty)
    assert np.array_equal(gpu.download().weight, w0)
    few = S.scan_patches(nx=3, ny=3, z=-0.12)           # 9 patches: patch 0 alone is sampled
    gpu.map_match(few)
    orc.map_match(few)
    assert_bit_identical(gpu.download(), orc.download(), "9-patch match")
    bad = S.scan_patches(nx=2, ny=2)
    bad[1].position[2] = float("nan")
    w1 = gpu.download().weight.copy()
    with pytest.raises(gpu_mod.EslamError):
        gpu.map_match(bad)
    assert np.array_equal(gpu.download().weight, w1)
    shared = gpu_mod.GpuFilter(S.bench_config(A.default_config(), n))
    so = O.OracleFilter(S.bench_config(A.default_config(), n), O.SUM_CONTRACT)
    for f in (shared, so):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
        f.step(S.step_stream(1)[0])
        f.map_match(S.scan_patches(x0=-0.3, x1=0.9))      # half on the grid's cells (x < 0.3)
    assert_bit_identical(shared.download(), so.download(), "shared-map match")
    shared.close()


@pytest.mark.parametrize("case", ["flat", "rough", "rough_heights", "rotated_grid"])
def test_shared_map_match_bit_exact(gpu_mod, oracle, case):
    """processMap(scanMap, match = true) with the shared map (useSharedMap = true: the laser
    path's match-only call, src/EmbodiedSlamFilter.cpp:214-221,342-344): every 10th patch
    scored against the patch getPatch's 3-sigma gate picks in the grid cell it lands on (0 when
    none passes; the rule is the build's own), weights feeding the resample of the
    next step.  Multi-patch cells (rough), vertical patches (heights) and a rotated grid; bit for
    bit against the oracle after every call."""
    n = 5003
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    grid = S.flat_map(cells=120) if case == "flat" else S.rough_map(cells=120)
    if case == "rough_heights":
        rng = np.random.default_rng(3)
        grid.patch_height = np.where(rng.random(grid.mean.shape[0]) < 0.3, rng.uniform(0.05, 0.5, grid.mean.shape[0]),
                                     0.0).astype(np.float32)
    if case == "rotated_grid":
        grid = rotated(grid)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.05], 0.18, 0.05)
    scans = [S.scan_patches(nx=12, ny=9, x0=-1.0, x1=2.5, y0=-1.5, y1=1.2, z=z) for z in (-0.18, -0.1, 0.4)]
    changed = 0
    for k, st in enumerate(S.step_stream(8, tilt=case != "flat")):
        assert gpu.step(st) == orc.step(st)
        w0 = gpu.download().weight.copy()
        gpu.map_match(scans[k % 3])
        orc.map_match(scans[k % 3])
        assert_bit_identical(gpu.download(), orc.download(), f"{case} shared match step {k}")
        changed += int(np.sum(gpu.download().weight != w0))
    assert np.array_equal(gpu.ancestors(), orc.ancestors())
    assert changed > n


@pytest.mark.parametrize("trail,n", [(16, 4096), (3, 1024)])
def test_particle_maps_loop_trail(gpu_mod, oracle, trail, n):
    """A loop: 6 m out and (nearly) back on the empty prior, a map update after every step.  The
    tiles each window leaves go to its trail and come back when the window returns (the
    reference's MLSMap keeps every grid, src/EmbodiedSlamFilter.cpp:195-207): on the way back the
    feet stand on the cells mapped on the way out (the scan looks ahead in +x, so it never maps
    them itself).  Bit-exact against the oracle (every particle, the counters of every update,
    the maps of sampled particles, trails included); a 3-entry trail overflows and forgets the
    farthest tiles, counted alike."""
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_PARTICLE_MAPS | A.FLAG_RECORD_ANCESTORS
    cfg.local_map_trail = trail
    cfg.local_map_pages = 32
    grid = S.unmapped_beyond(S.flat_map(cells=200), -1e9)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_threads(16)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    scan = S.scan_patches()
    stream = S.step_stream(300, dx=0.02, dyaw=0.0) + S.step_stream(260, dx=-0.02, dyaw=0.0)
    evicted, found = 0, []
    for k, st in enumerate(stream):
        assert gpu.step(st) == orc.step(st)
        gpu.map_update(scan)
        orc.map_update(scan)
        gi = gpu.sync()
        assert map_info(gi) == map_info(orc.info()), (k, map_info(gi), map_info(orc.info()))
        evicted += gi.map_tiles_evicted
        if k >= 300:
            found.append(gi.data_particles / n)
        if k % 80 == 79 or k == len(stream) - 1:
            assert_bit_identical(gpu.download(), orc.download(), f"loop trail={trail} step {k}")
            assert_maps_equal(gpu, orc, [0, 1, n // 2, n - 1], f"loop step {k}")
    assert np.array_equal(gpu.ancestors(), orc.ancestors())
    if trail == 16:
        assert evicted == 0
        assert np.mean(found[-80:]) > 0.9, found[-80:]       # on the cells of the way out
    else:
        assert evicted > 0
