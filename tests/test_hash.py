"""SurfaceHash (useHash = true) in the CPU oracle: the glibc rand() restatement, the pose
hash of SurfaceHash::create against an independent numpy restatement, and the respawn of
PoseEstimator::sampleFromHash (src/SurfaceHash.hpp:155-231, src/PoseEstimator.cpp:75-86,
130-182)."""
import ctypes as C
import ctypes.util
import math

import numpy as np
import pytest

import eslam_abi as A
import oracle_ffi as O
import synthetic as S
from hash_util import hash_config, hash_grid, rotated_grid, slope_stream


def test_libc_rand_matches_glibc(oracle):
    """dm_libc_rand == this system's rand() after srand(1) (the reference's unseeded rand())."""
    libc = C.CDLL(ctypes.util.find_library("c"))
    libc.srand(1)
    want = [libc.rand() for _ in range(5000)]
    got = (C.c_int32 * 5000)()
    oracle.lib().or_dm_libc_rand(1, 5000, got)
    assert list(got) == want


def numpy_hash(grid, steps, bins):
    """Independent restatement of SurfaceHash::create (numpy least squares for the plane)."""
    W, H = grid.width, grid.height
    sx, sy = grid.scale
    ox, oy = grid.offset
    feet = np.array([[0.25, 0.0], [-0.25, 0.0], [0.25, -0.5], [-0.25, -0.5]])
    ang = 2 * math.pi / steps
    R = np.array([[math.cos(ang), -math.sin(ang)], [math.sin(ang), math.cos(ang)]])
    pts = feet.copy()
    first = grid.mean[grid.cell_start[:-1].clip(max=len(grid.mean) - 1)]
    has = grid.cell_start[1:] > grid.cell_start[:-1]
    out = []
    for a in range(steps):
        pts = pts @ R.T
        for m in range(W):
            for n in range(H):
                x, y = (m + 0.5) * sx + ox, (n + 0.5) * sy + oy
                gp = []
                for i in range(4):
                    fm = math.floor(((x + pts[i, 0]) - ox) * (1 / sx))
                    fn = math.floor(((y + pts[i, 1]) - oy) * (1 / sy))
                    if 0 <= fm < W and 0 <= fn < H and has[fn * W + fm]:
                        gp.append((feet[i, 0], feet[i, 1], float(first[fn * W + fm])))
                if len(gp) < 3:
                    continue
                P = np.array(gp)
                coef, *_ = np.linalg.lstsq(np.c_[P[:, 0], P[:, 1], np.ones(len(P))], P[:, 2], rcond=None)
                bx = min(bins - 1, max(0, int((coef[0] + 1) / 2 * bins)))
                by = min(bins - 1, max(0, int((coef[1] + 1) / 2 * bins)))
                out.append((x, y, a * 2 * math.pi / steps, P[:, 2].mean() + 0.18, bx * bins + by, coef[0], coef[1]))
    return out


def test_hash_create_against_numpy(oracle):
    grid = hash_grid(cells=24)
    cfg = hash_config(100, steps=4, bins=20)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(grid)
    f.hash_create()
    x, y, th, z, bucket = f.hash_poses()
    want = numpy_hash(grid, 4, 20)
    assert len(want) == len(x) > 100
    for k, (wx, wy, wth, wz, wb, slx, sly) in enumerate(want):
        assert abs(x[k] - wx) < 1e-12 and abs(y[k] - wy) < 1e-12 and abs(th[k] - wth) < 1e-12
        assert abs(z[k] - wz) < 1e-9
        # the bucket agrees unless the slope sits on a bin edge (LDLT vs lstsq rounding)
        edge = min(abs((slx + 1) / 2 * 20 - round((slx + 1) / 2 * 20)), abs((sly + 1) / 2 * 20 - round((sly + 1) / 2 * 20)))
        assert bucket[k] == wb or edge < 1e-9
    n, sizes = f.hash_info()
    assert n == len(x) and sizes.sum() == n


def test_hash_flat_map_single_bucket(oracle):
    cfg = hash_config(100, steps=4, bins=20)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(S.flat_map(cells=20))
    f.hash_create()
    n, sizes = f.hash_info()
    assert n > 0 and sizes[10 * 20 + 10] == n        # slope 0 -> bucket (10, 10)


def test_hash_rotated_grid_frame(oracle):
    """grid2world = inverse(global2local) places the poses and offsets their yaw."""
    cfg = hash_config(100, steps=4, bins=20)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(rotated_grid(cells=20))
    f.hash_create()
    x, y, th, z, _ = f.hash_poses()
    assert np.allclose(np.unique(np.round(th, 9)) - 0.3, np.arange(4) * math.pi / 2, atol=1e-9)


def test_init_hash_and_respawn(oracle):
    n = 3000
    cfg = hash_config(n, steps=8, bins=20, period=2)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_map(hash_grid())
    f.init_pose([0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0])
    pa = f.download()
    assert np.all(pa.zsigma == 0.0) and np.all(pa.floating == 1) and np.all(pa.weight == 0.0)
    hx, hy, hth, hz, _ = f.hash_poses()
    poses = set(zip(hx.tolist(), hy.tolist()))
    assert all((a, b) in poses for a, b in zip(pa.x[:200].tolist(), pa.y[:200].tolist()))
    st = slope_stream(5)
    replaced = 0
    for k, s in enumerate(st):
        f.project(s)
        pa = f.download()
        if k % 2 == 0:          # the respawn step (first project, then every period-th)
            replaced = max(replaced, int(np.count_nonzero(pa.zsigma == 0.5)))
        f.update(s)
    assert replaced > 0, "the slope feet should select a rare bucket and replace particles"
