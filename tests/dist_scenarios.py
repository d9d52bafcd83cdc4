"""Scenarios shared by the multi-rank tests (test infrastructure).

``run_scenario`` drives one filter -- the whole filter (lo=0, hi=n_global) or one rank's
shard [lo, hi) of it -- through a fixed sequence of inputs and records everything the
rank holds after every call.  A sharded run concatenated over the ranks must equal the
single run bit for bit (include/eslam_gpu.h, eslam_gpu_set_comm)."""
import numpy as np

import eslam_abi as A
import synthetic as S

FIELDS = ("x", "y", "orientation", "zpos", "zsigma", "weight", "mprob", "floating", "n_contact_points")
SCENARIOS = ("forced", "natural", "upload", "hash", "config3", "config4", "maps", "edit", "records", "heirloom", "chunks")
EDIT_GLOBAL = (0, 37)                            # edit: the particles one rank edits
CONFIG3_STEPS = 3
MAP_SAMPLES = 64                                 # config4: particles whose maps are compared
RECORD_CPOINTS = 8                               # records: contact points per particle compared


def scenario_config(name, n_global):
    if name == "hash":                           # useHash: init from the hash, respawn every 2nd step
        from hash_util import hash_config
        cfg = hash_config(n_global, steps=8, bins=20, period=2, percentage=0.2)
        cfg.seed = 1234
        return cfg
    cfg = A.default_config()
    cfg.seed = 1234
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    if name in ("forced", "config3", "config4", "maps", "burst", "edit", "getter0", "records", "heirloom", "chunks"):
        S.bench_config(cfg, n_global)
        if name == "chunks":                     # an explicit summation chunk (eslam_config.sum_chunk_rows)
            cfg.sum_chunk_rows = 3
        if name == "config3":
            # the chunk a sharded configs[3] uses: sized by the 2M of one of its 8 ranks (7 rows),
            # so that each rank's weighting kernel fills the chip (13 rows from the 16M would
            # leave half of it idle: K1 +24 % per rank, profiles/r06/ab/ab_r06r_chunk_rows.log)
            cfg.sum_chunk_rows = A.chunk_rows(-(-n_global // 8))
        if name == "records":                    # logDebug: every update's contact points
            cfg.flags |= A.FLAG_RECORD_CONTACTS
        if name in ("maps", "config4", "heirloom"):   # useSharedMap = false: per-particle maps
            cfg.flags |= A.FLAG_PARTICLE_MAPS
        if name == "heirloom":
            # 8 pages per particle: the one map of ~50 pages fits the pool once, not once per copy
            # (then a map update's copies on write take ~4 per particle)
            cfg.local_map_pages = 8
        if name == "config4":
            # 8 ranks x 8M and then one 64M context share one GPU's 288 GB: a 5 x 5-tile window
            # (1.5 m; the scan reaches 1.2 m) and 6 pages per particle (3 steps take ~5)
            cfg.max_sensor_range = 1.5
            cfg.local_map_pages = 6
    else:
        cfg.particle_count = n_global
        cfg.min_effective = (n_global * 9) // 10
        cfg.measurement_threshold_distance = -1.0
        cfg.measurement_threshold_angle = -1.0
    return cfg


def scenario_grid(name):
    if name == "hash":
        from hash_util import hash_grid
        return hash_grid(cells=60)
    if name == "config3":
        return S.flat_map(cells=1000)             # the bench's 100 x 100 m map
    if name == "config4":                         # bench.py --local-maps: rough, scans map x > 0.3 m
        return S.unmapped_beyond(S.rough_map(cells=1000), 0.3)
    if name == "maps":                            # the front feet stand on cells only the scans map
        return S.unmapped_beyond(S.rough_map(cells=120), 0.3)
    if name == "heirloom":                        # the empty prior: every cell is a particle's own
        return S.unmapped_beyond(S.rough_map(cells=120), -1e9)
    return S.rough_map(cells=120) if name not in ("forced", "burst", "edit", "getter0", "records") else S.rough_map(cells=120, multi=False)


def digest(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()


def map_samples(n_global):
    """global indices of the particles whose maps config4 compares"""
    return sorted(set(np.linspace(0, n_global - 1, MAP_SAMPLES).astype(np.int64).tolist()))


def run_config3(f, n_global, lo, hi, info_fn, name="config3"):
    """BASELINE configs[3]'s workload (bench map, forced update + resample, init as the bench)
    for CONFIG3_STEPS steps; records per-step info and, at the end, a SHA-256 of every field of
    this shard / slice [lo, hi) and of the last step's ancestors (a 16M-particle snapshot is
    too large to ship between processes).  name="config4": configs[4]'s workload instead --
    per-particle maps on the rough map unmapped beyond x = 0.3 m, tilted body, one scan merged
    after every step -- plus the SHA-256 of the maps of map_samples() in [lo, hi)."""
    rec = {}
    maps = name == "config4"
    f.set_map(scenario_grid(name))
    f.init_gaussian(hi - lo, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    scan = S.scan_patches() if maps else None
    for k, st in enumerate(S.step_stream(CONFIG3_STEPS, tilt=maps)):
        f.step(st)
        if maps:
            f.map_update(scan)
        _info(rec, f"s{k}", info_fn(f))
    if maps:
        for g in map_samples(n_global):
            if lo <= g < hi:
                c, m, s = f.particle_map(g - lo)
                o = np.argsort(c)
                rec[f"map/{g}"] = np.array(digest(np.concatenate([c[o].view(np.uint8), m[o].view(np.uint8),
                                                                  s[o].view(np.uint8)])))
    pa = f.download()
    anc = f.ancestors()
    best, rng = np.array([f.best_index()]), np.array([f.rng_state().minstd_x])
    pos, quat = f.centroid()
    rec["centroid"] = np.array(list(pos) + list(quat))
    return rec, {fld: np.array(getattr(pa, fld)) for fld in FIELDS}, np.asarray(anc), best, rng


def upload_arrays(n_global, lo, hi):
    rng = np.random.default_rng(99)
    pa = A.ParticleArrays(n_global)
    pa.x[:] = rng.normal(0, 0.2, n_global)
    pa.y[:] = rng.normal(0, 0.2, n_global)
    pa.orientation[:] = rng.normal(0, 0.1, n_global)
    pa.zpos[:] = 0.18 + rng.normal(0, 0.01, n_global)
    pa.zsigma[:] = 0.5
    w = rng.exponential(1.0, n_global) ** 3
    w[rng.random(n_global) < 0.2] = 0.0
    pa.weight[:] = w
    pa.mprob[:] = 1.0
    pa.floating[:] = 1
    pa.n_contact_points[:] = 0
    out = A.ParticleArrays(hi - lo)
    for f in FIELDS:
        getattr(out, f)[:] = getattr(pa, f)[lo:hi]
    return out


def _snap(rec, key, f, with_anc):
    pa = f.download()
    for fld in FIELDS:
        rec[f"{key}/{fld}"] = np.array(getattr(pa, fld))
    if with_anc:
        rec[f"{key}/anc"] = f.ancestors()


def _info(rec, key, i):
    rec[f"{key}/info"] = np.array([i.effective, i.weight_sum, i.floating_weight, i.max_weight,
                                   float(i.data_particles), float(i.total_points), float(i.resampled),
                                   float(i.uniform_reset)])


def edit_particles(f, lo, hi):
    """the caller edits particles through getParticles() (processMap's weights,
    src/EmbodiedSlamFilter.cpp:183-220): global EDIT_GLOBAL, which lie on the first rank only.
    A GPU filter writes them back with eslam_gpu_write_particles -- a collective on a sharded
    filter, which every rank calls (the others with nothing to write); the oracle replaces its
    shard (download, edit, upload: the same particles, documented in include/eslam_gpu.h)."""
    g0, g1 = max(EDIT_GLOBAL[0], lo), min(EDIT_GLOBAL[1], hi)
    pa = f.download()
    if g1 > g0:
        sl = slice(g0 - lo, g1 - lo)
        pa.weight[sl] = pa.weight[sl] * 3.5 + 0.25       # above 1: the weight scale changes
        pa.x[sl] = pa.x[sl] + 0.01
    if hasattr(f, "write"):
        part = A.ParticleArrays(max(g1 - g0, 0))
        for fld in FIELDS:
            if g1 > g0:
                getattr(part, fld)[:] = getattr(pa, fld)[g0 - lo:g1 - lo]
        f.write(g0 - lo if g1 > g0 else 0, part)
    else:
        f.upload(pa)


def _records(rec, key, f):
    """logDebug's PoseParticle records (eslam_gpu_download_records: cpoints, meas_pos,
    meas_theta of each particle's ancestor at the last update; a collective on a sharded
    filter, so every rank calls it)"""
    r, cps = f.download_records(max_cpoints=RECORD_CPOINTS)
    for fld in ("index", "n_cpoints", "meas_pos", "meas_theta", "position", "weight"):
        rec[f"{key}/rec_{fld}"] = np.ascontiguousarray(r[fld])
    for fld in ("point", "zdiff", "zvar", "prob"):
        rec[f"{key}/cp_{fld}"] = np.ascontiguousarray(cps[fld])


def heirloom_arrays(n_global, lo, hi):
    """every particle off the grid (x = 1000 m) with weight 0 but the last one: at the origin,
    weight 1 -- its map is the only one, and a resample copies it to every output"""
    pa = A.ParticleArrays(hi - lo)
    pa.x[:] = 1000.0
    pa.zpos[:] = 0.18
    pa.zsigma[:] = 0.05
    pa.mprob[:] = 1.0
    pa.floating[:] = 1
    if hi == n_global:
        pa.x[-1] = 0.0
        pa.weight[-1] = 1.0
    return pa


def _maps(rec, f, n):
    """every particle's own patches, sorted by cell"""
    count = np.zeros(n, np.uint32)
    cells, mean, sd = [], [], []
    for i in range(n):
        c, m, s_ = f.particle_map(i)
        o = np.argsort(c)
        count[i] = len(c)
        cells.append(c[o]); mean.append(m[o]); sd.append(s_[o])
    rec["maps/count"] = count
    rec["maps/cells"] = np.concatenate(cells) if cells else np.zeros(0, np.uint32)
    rec["maps/mean"] = np.concatenate(mean) if mean else np.zeros(0, np.float32)
    rec["maps/stdev"] = np.concatenate(sd) if sd else np.zeros(0, np.float32)


def run_scenario(f, name, n_global, lo, hi, steps=6, info_fn=None):
    """f: OracleFilter or GpuFilter-like (set_map/init_gaussian/upload/step/...).
    info_fn(f) returns the eslam_update_info of the last update."""
    rec = {}
    grid = scenario_grid(name)
    f.set_map(grid)
    if name == "heirloom":
        # one particle on the last rank maps a wide scan (~50 pages) and then holds all the weight:
        # the resample copies it to every output, so every other rank receives one record for
        # all its particles (one table and one set of pages for the record, not one per copy),
        # and map updates then copy on write what each particle changes.  (A resample that
        # migrates many records deep-copies each record's pages: pages two records shared on
        # the sending rank are two copies on the receiving one.)
        f.upload(heirloom_arrays(n_global, lo, hi))
        f.map_update(S.scan_patches(nx=16, ny=12, x0=-2.6, x1=4.6, y0=-2.5, y1=2.4))
        f.resample()
        _snap(rec, "res", f, True)
        _maps(rec, f, hi - lo)
        for k in range(2):                       # the copies on write of the shared received table
            f.map_update(S.scan_patches(x0=0.35 + 0.3 * k))
        rec["maps2/count"] = np.array([len(f.particle_map(g - lo)[0]) for g in range(lo, hi) if g % 97 == 0], np.uint32)
        return rec
    if name == "upload":
        f.upload(upload_arrays(n_global, lo, hi))
        rec["sum0"] = np.array([f.weights_sum()])
        rec["best0"] = np.array([f.best_index()])
        rec["eff0"] = np.array([f.normalize()])
        _snap(rec, "norm", f, False)
        f.resample()
        _snap(rec, "res", f, True)
    elif name == "hash":
        f.init_pose([0.0, 0.0, 0.18], [1.0, 0.0, 0.0, 0.0])       # SurfaceHash::create + init(N, hash)
    elif name == "maps":
        f.init_gaussian(hi - lo, [0.0, 0.0, 0.0], [0.05, 0.05, 0.02], 0.18, 0.05)
    else:
        sigma = [0.1, 0.1, 0.1] if name == "forced" else [0.6, 0.6, 0.3]
        f.init_gaussian(hi - lo, [0.0, 0.0, 0.0], sigma, 0.18, 1.001)
    if name == "getter0":
        # forced updates back to back, then only the first rank reads its particles (a
        # rank-local getter, which completes the last update's deferred exchange on a sharded
        # GPU filter) and every rank closes its filter: close() runs the collective
        # eslam_gpu_finish, which completes the exchange on the other ranks, so no rank is
        # left waiting in it (destroy itself never communicates)
        for st in S.step_stream(steps):
            f.step(st)
        if lo == 0:
            _snap(rec, "last", f, True)
        return rec
    if name == "burst":
        # forced updates back to back with nothing read between them: a sharded GPU filter
        # defers each update's exchange into the next step (split weighting launch)
        for st in S.step_stream(steps):
            f.step(st)
        _info(rec, "last", info_fn(f))
        _snap(rec, "last", f, True)
        rec["best"] = np.array([f.best_index()])
        rec["rng"] = np.array([f.rng_state().minstd_x])
        return rec
    _snap(rec, "init", f, False)
    if name == "hash":
        from hash_util import slope_stream
        stream = slope_stream(steps)
    else:
        stream = S.step_stream(steps, tilt=(name in ("natural", "maps")))
    scan = S.scan_patches() if name == "maps" else None
    probe = S.scan_patches(z=-0.15) if name == "maps" else None
    for k, st in enumerate(stream):
        if name == "edit" and k == 2:
            edit_particles(f, lo, hi)
            _snap(rec, "edit", f, False)
        f.step(st)
        info = info_fn(f)
        _info(rec, f"s{k}", info)
        _snap(rec, f"s{k}", f, bool(info.resampled))
        if name == "records":
            _records(rec, f"s{k}", f)
        if scan is not None and k % 2 == 1:      # processMap(probe, true, ...): the match weighting
            f.map_match(probe)
            _snap(rec, f"m{k}", f, False)
        if scan is not None:                     # processMap(scan, false, true)
            f.map_update(scan)
    if scan is not None:                         # every particle's own patches, sorted by cell
        _maps(rec, f, hi - lo)
    rec["best"] = np.array([f.best_index()])
    rec["rng"] = np.array([f.rng_state().minstd_x])
    pos, quat = f.centroid()                 # getCentroid (normalises in place, Q15)
    rec["centroid"] = np.array(list(pos) + list(quat))
    _snap(rec, "centroid", f, False)
    return rec
