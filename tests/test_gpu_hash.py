"""SurfaceHash on the GPU against the oracle, bit for bit: the pose hash of
SurfaceHash::create (sweep kernel), PoseEstimator::init(N, hash) and the sampleFromHash
respawn inside the step (radix sort of the (float weight, index) pairs on the device)."""
import numpy as np
import pytest

import oracle_ffi as O
from hash_util import hash_config, hash_grid, rotated_grid, slope_stream
from parity_util import assert_bit_identical, info_tuple

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("grid_fn", [hash_grid, rotated_grid])
def test_hash_create_parity(gpu_mod, grid_fn):
    grid = grid_fn(cells=60)
    cfg = hash_config(1000, steps=8, bins=20)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    gpu = gpu_mod.GpuFilter(cfg)
    for f in (orc, gpu):
        f.set_map(grid)
        f.hash_create()
    no, so = orc.hash_info()
    ng, sg = gpu.hash_info()
    assert no == ng > 0 and np.array_equal(so, sg)
    for a, b in zip(gpu.hash_poses(), orc.hash_poses()):
        assert np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


@pytest.mark.parametrize("mode", ["step", "split"])
def test_hash_filter_parity(gpu_mod, mode):
    n = 5000
    cfg = hash_config(n, steps=8, bins=20, period=2)
    grid = hash_grid(cells=60)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    gpu = gpu_mod.GpuFilter(cfg)
    for f in (orc, gpu):
        f.set_map(grid)
        f.init_pose([0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0])
    assert_bit_identical(gpu.download(), orc.download(), "init from hash")
    replaced = 0
    for k, st in enumerate(slope_stream(7)):
        if mode == "step":
            orc.step(st)
            gpu.step(st)
        else:
            orc.project(st)
            gpu.project(st)
            pa = gpu.download()
            assert_bit_identical(pa, orc.download(), f"project {k}")
            replaced += int(np.count_nonzero(pa.zsigma == 0.5))
            orc.update(st)
            gpu.update(st)
        gi = gpu.sync()
        assert_bit_identical(gpu.download(), orc.download(), f"{mode} step {k}")
        assert info_tuple(gi) == info_tuple(orc.info()), k
    if mode == "split":
        assert replaced > 0
    assert gpu.rng_state().libc_rand_pos == orc.rng_state().libc_rand_pos


@pytest.mark.parametrize("n,distinct", [(1, 4), (1000, 3), (2048 * 3 + 17, 50), (1 << 20, 1 << 31)])
def test_radix_sort_stable(gpu_mod, n, distinct):
    """The hand-written radix sort behind sampleFromHash's (float weight, index) order: equal
    to numpy's stable argsort, many-way ties included (the respawn's draws follow this order)."""
    import ctypes as C
    rng = np.random.default_rng(n)
    keys = rng.integers(0, distinct, n, dtype=np.uint64).astype(np.uint32) * np.uint32(0x9E3779B1)
    vals = np.arange(n, dtype=np.uint32)
    ko = np.zeros(n, np.uint32)
    vo = np.zeros(n, np.uint32)
    L = gpu_mod.load_library()
    p = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32))
    assert L.eslam_gpu_selftest_sort(0, p(keys), p(vals), n, p(ko), p(vo)) == 0
    order = np.argsort(keys, kind="stable")
    assert np.array_equal(vo, vals[order]) and np.array_equal(ko, keys[order])
