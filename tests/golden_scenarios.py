"""Scenarios of the golden vectors (tests/golden/) -- test infrastructure."""
import numpy as np

import eslam_abi as A
import synthetic as S

N = 512
STEPS = 4
FIELDS = ("x", "y", "orientation", "zpos", "zsigma", "weight", "mprob", "floating", "n_contact_points")
SCENARIOS = ("flat_forced", "rough_natural", "grouped_nan", "hash_slope")


def setup(name):
    cfg = A.default_config()
    cfg.seed = 2024
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    cfg.particle_count = N
    init = dict(mu=[0.0, 0.0, 0.0], sigma=[0.1, 0.1, 0.1], z=0.18, zs=1.001)
    if name == "flat_forced":
        S.bench_config(cfg, N)
        grid, stream = S.flat_map(cells=100), S.step_stream(STEPS)
    elif name == "rough_natural":
        cfg.min_effective = N // 2
        cfg.measurement_threshold_distance = -1.0
        cfg.measurement_threshold_angle = -1.0
        grid, stream = S.rough_map(cells=100), S.step_stream(STEPS, tilt=True)
        init = dict(mu=[0.0, 0.0, 0.0], sigma=[0.5, 0.5, 0.3], z=0.18, zs=1.001)
    elif name == "grouped_nan":
        feet = [(0.3, 0.1, -0.18), (0.3, -0.1, -0.2), (-0.3, 0.1, -0.18), (-0.3, -0.1, -0.22),
                (0.3, -0.5, -0.18), (0.3, -0.7, -0.19), (-0.3, -0.5, -0.18), (-0.3, -0.7, -0.25)]
        contact = lambda s, i: float("nan") if (s + i) % 3 == 0 else (0.1 if (s * 7 + i) % 5 == 0 else 0.9)
        cfg.min_contacts = 2
        grid = S.rough_map(cells=100)
        stream = S.step_stream(STEPS, tilt=True, feet=feet, groups=[0, 0, 1, 1, 2, 2, 3, 3], contact=contact, ltc=1)
        init = dict(mu=[0.0, 0.0, 0.0], sigma=[2.0, 2.0, 1.0], z=0.18, zs=0.3)
    elif name == "hash_slope":
        from hash_util import hash_config, hash_grid, slope_stream
        cfg = hash_config(N, steps=8, bins=20, period=2, percentage=0.2)
        cfg.seed = 2024
        grid, stream = hash_grid(cells=60), slope_stream(STEPS)
        init = "pose"
    else:
        raise KeyError(name)
    return cfg, grid, stream, init


def snapshot(rec, key, f, anc):
    pa = f.download()
    for fld in FIELDS:
        rec[f"{key}/{fld}"] = np.array(getattr(pa, fld))
    if anc:
        rec[f"{key}/anc"] = np.array(f.ancestors())


def run(name, make, info_fn):
    cfg, grid, stream, init = setup(name)
    f = make(cfg)
    f.set_map(grid)
    if init == "pose":
        f.init_pose([0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0])
    else:
        f.init_gaussian(N, init["mu"], init["sigma"], init["z"], init["zs"])
    rec = {}
    snapshot(rec, "init", f, False)
    for k, st in enumerate(stream):
        f.step(st)
        i = info_fn(f)
        rec[f"s{k}/info"] = np.array([i.effective, i.weight_sum, i.floating_weight, i.max_weight, float(i.data_particles),
                                      float(i.total_points), float(i.resampled), float(i.uniform_reset),
                                      float(i.resample_overruns)])
        snapshot(rec, f"s{k}", f, bool(i.resampled))
    r = f.rng_state()
    rec["rng"] = np.array([r.minstd_x, r.project_count, r.init_count, r.hash_count, r.libc_rand_pos], dtype=np.uint64)
    return rec
