"""Synthetic inputs for the eSLAM hot path (BASELINE.md "Synthetic inputs").

The reference ships no datasets; its only numeric harness (test/testMap.cpp) is seeded with
time(0).  These generators produce the deterministic map + odometry/foot-contact stream the
benchmarks and parity tests run on:

* flat map   : 1000 x 1000 cells @ 0.1 m (100 x 100 m, origin (-50, -50)), one horizontal
               patch per cell, mean 0, stdev 0.05                         (configs 1-4)
* rough map  : sum of 3 sinusoids (amplitude 0.2 m, wavelengths 1-5 m) + N(0, 0.02) noise,
               1 patch per cell w.p. 0.6 else 2-8 patches separated by >= 1.5 m gaps,
               stdev ~ U(0.02, 0.1), seed 7                               (config 5)
* stream     : per step delta = (0.02 m, 0, 0.002 rad), Sigma = diag(1e-4, 1e-4, 1e-5),
               4 feet at (+-0.25, 0, -0.18), (+-0.25, -0.5, -0.18), contact 1, ungrouped.
* mapping    : (config 5's per-particle local maps) the map without its cells beyond x0
               (terrain the robot has not mapped yet) and a scan of the ground ahead of the
               robot, 8 x 6 patches in the yaw-free body frame.
"""
import math

import numpy as np

from eslam_abi import GridArrays, StepInput, MAX_CONTACTS

FEET = [(0.25, 0.0, -0.18), (-0.25, 0.0, -0.18), (0.25, -0.5, -0.18), (-0.25, -0.5, -0.18)]


def flat_map(cells=1000, res=0.1, mean=0.0, stdev=0.05):
    half = cells * res / 2.0
    n = cells * cells
    cell_start = np.arange(n + 1, dtype=np.uint32)
    return GridArrays(cells, cells, (res, res), (-half, -half), cell_start,
                      np.full(n, mean, np.float32), np.full(n, stdev, np.float32))


def rough_map(cells=1000, res=0.1, seed=7, multi=True):
    rng = np.random.default_rng(seed)
    half = cells * res / 2.0
    xs = -half + (np.arange(cells) + 0.5) * res
    X, Y = np.meshgrid(xs, xs, indexing="xy")          # Y varies along rows (n), X along m
    amp = 0.2 / 3.0
    ground = (amp * np.sin(2 * math.pi * X / 1.0 + 0.3)
              + amp * np.sin(2 * math.pi * Y / 3.0 + 1.1)
              + amp * np.sin(2 * math.pi * (X + Y) / 5.0 + 2.0))
    ground = ground + rng.normal(0.0, 0.02, ground.shape)
    ground = ground.reshape(-1)                          # index n * width + m
    ncell = cells * cells
    if multi:
        k = np.where(rng.random(ncell) < 0.6, 1, rng.integers(2, 9, ncell))
    else:
        k = np.ones(ncell, dtype=np.int64)
    cell_start = np.zeros(ncell + 1, dtype=np.uint64)
    np.cumsum(k, out=cell_start[1:])
    total = int(cell_start[-1])
    owner = np.repeat(np.arange(ncell), k)
    rank = np.arange(total) - np.repeat(cell_start[:-1], k).astype(np.int64)
    gaps = 1.5 + rng.random(total)
    # stacked patches: level j sits j gaps above the ground patch (ascending mean)
    offs = np.zeros(total)
    if total:
        csum = np.cumsum(np.where(rank == 0, 0.0, gaps))
        base = np.repeat(csum[cell_start[:-1].astype(np.int64)], k)
        offs = csum - base
    mean = ground[owner] + offs
    stdev = rng.uniform(0.02, 0.1, total)
    return GridArrays(cells, cells, (res, res), (-half, -half), cell_start.astype(np.uint32),
                      mean.astype(np.float32), stdev.astype(np.float32))


def quat_from_rpy(roll, pitch, yaw):
    cr, sr = math.cos(roll / 2), math.sin(roll / 2)
    cp, sp = math.cos(pitch / 2), math.sin(pitch / 2)
    cy, sy = math.cos(yaw / 2), math.sin(yaw / 2)
    return (cr * cp * cy + sr * sp * sy,
            sr * cp * cy - cr * sp * sy,
            cr * sp * cy + sr * cp * sy,
            cr * cp * sy - sr * sp * cy)


def step_stream(steps, tilt=False, feet=FEET, contact=1.0, groups=None, z_delta=0.0,
                dx=0.02, dyaw=0.002, ltc=0):
    """List of StepInput for `steps` consecutive odometry steps."""
    out = []
    x = y = yaw = 0.0
    for s in range(steps):
        yaw += dyaw
        x += dx * math.cos(yaw)
        y += dx * math.sin(yaw)
        roll = 0.05 * math.sin(0.37 * s) if tilt else 0.0
        pitch = 0.04 * math.sin(0.23 * s + 0.5) if tilt else 0.0
        st = StepInput()
        st.body2odometry_rot[:] = quat_from_rpy(roll, pitch, yaw)
        st.body2odometry_trans[:] = [x, y, 0.0]
        st.pose_delta_trans[:] = [dx, 0.0, z_delta]
        st.position_error_zz = 1e-4
        st.sample_mean[:] = [dx, 0.0, dyaw]
        st.sample_cov[:] = [1e-4, 0, 0, 0, 1e-4, 0, 0, 0, 1e-5]
        st.n_contacts = len(feet)
        st.ltc_count = ltc
        for i, f in enumerate(feet):
            st.contacts[i].position[:] = list(f)
            st.contacts[i].contact = contact if not callable(contact) else contact(s, i)
            st.contacts[i].group_id = -1 if groups is None else groups[i]
        out.append(st)
    assert len(feet) <= MAX_CONTACTS
    return out


def bench_config(cfg, n):
    """Benchmark configuration: N particles, resample forced every step (minEffective = N+1),
    measurement update forced (thresholds below any motion)."""
    cfg.particle_count = n
    cfg.min_effective = n + 1
    cfg.measurement_threshold_distance = -1.0
    cfg.measurement_threshold_angle = -1.0
    return cfg


def unmapped_beyond(grid, x0):
    """The grid with no patches in the cells whose centre lies at x >= x0 (unmapped terrain)."""
    w, h = grid.width, grid.height
    xc = grid.offset[0] + (np.arange(w) + 0.5) * grid.scale[0]
    keep_cell = np.tile(xc < x0, h)                              # cell n * w + m
    counts = np.diff(grid.cell_start.astype(np.int64))
    keep_patch = np.repeat(keep_cell, counts)
    new_counts = np.where(keep_cell, counts, 0)
    cell_start = np.zeros(w * h + 1, dtype=np.uint64)
    np.cumsum(new_counts, out=cell_start[1:])
    ph = None if grid.patch_height is None else grid.patch_height[keep_patch]
    return GridArrays(w, h, grid.scale, grid.offset, cell_start.astype(np.uint32), grid.mean[keep_patch],
                      grid.stdev[keep_patch], ph, grid.g2l)


def scan_patches(nx=8, ny=6, x0=0.35, x1=0.95, y0=-0.7, y1=0.2, z=-0.18, stdev=0.03):
    """A scan of the ground ahead: nx x ny patches (x, y, z, stdev) in the yaw-free body
    frame (the cells of processMap's scan MLS), with a gentle height pattern."""
    import eslam_abi as A
    out = (A.ScanPatch * (nx * ny))()
    k = 0
    for i in range(nx):
        for j in range(ny):
            x = x0 + (x1 - x0) * i / max(nx - 1, 1)
            y = y0 + (y1 - y0) * j / max(ny - 1, 1)
            out[k].position[:] = [x, y, z + 0.01 * math.sin(3.0 * x + 2.0 * y)]
            out[k].stdev = stdev
            k += 1
    return out


def scan_area(count, nx=25, spacing=0.1, x0=0.35, yc=-0.25, z=-0.18, stdev=0.03):
    """A laser scan's MLS ahead of the robot at the map's resolution: `count` patches on a grid
    of nx columns (x0 .. x0 + (nx - 1) spacing ahead) and ceil(count / nx) rows centred on yc,
    in the yaw-free body frame (600 patches: 2.5 m x 2.4 m at 0.1 m, within maxSensorRange 3 m,
    src/Configuration.hpp:107)."""
    import eslam_abi as A
    ny = -(-count // nx)
    out = (A.ScanPatch * count)()
    k = 0
    for i in range(nx):
        for j in range(ny):
            if k == count:
                break
            x = x0 + spacing * i
            y = yc + spacing * (j - (ny - 1) / 2.0)
            out[k].position[:] = [x, y, z + 0.01 * math.sin(3.0 * x + 2.0 * y)]
            out[k].stdev = stdev
            k += 1
    return out

