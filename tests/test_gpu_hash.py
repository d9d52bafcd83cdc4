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


def _share(src, dst):
    """the process-wide statics of src (hash counter, rand()) handed to dst's oracle"""
    s, t = dst.rng_state(), src.rng_state()
    s.hash_count = t.hash_count
    s.libc_rand[:] = t.libc_rand[:]
    s.libc_rand_pos = t.libc_rand_pos
    dst.set_rng_state(s)


def test_process_statics_shared_between_contexts(gpu_mod):
    """Q11 (ESLAM_FLAG_PROCESS_STATICS): two filters of one process share the function-static
    hash-respawn counter (src/PoseEstimator.cpp:239) and rand(), as the reference's do.  Two
    flagged contexts stepped in turn equal two oracle filters that hand the counter and the
    rand() state to each other before every call, bit for bit; the counter then counts both."""
    import eslam_abi as A
    n = 2000
    cfg = hash_config(n, steps=8, bins=20, period=3)
    cfg.flags |= A.FLAG_PROCESS_STATICS
    grid = hash_grid(cells=60)
    ga, gb = gpu_mod.GpuFilter(cfg), gpu_mod.GpuFilter(cfg)
    oa, ob = O.OracleFilter(cfg, O.SUM_CONTRACT), O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (ga, gb, oa, ob):
        f.set_map(grid)
    h0 = ga.rng_state().hash_count
    ga.init_pose([0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0])
    oa.init_pose([0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0])
    _share(oa, ob)
    gb.init_pose([0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0])
    ob.init_pose([0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0])
    steps = slope_stream(5)
    for k, st in enumerate(steps):
        _share(ob, oa)
        ga.step(st)
        oa.step(st)
        _share(oa, ob)
        gb.step(st)
        ob.step(st)
        assert_bit_identical(ga.download(), oa.download(), f"A step {k}")
        assert_bit_identical(gb.download(), ob.download(), f"B step {k}")
    sa, sb = ga.rng_state(), gb.rng_state()
    assert sa.hash_count == sb.hash_count == h0 + 2 * len(steps)
    assert sa.libc_rand_pos == sb.libc_rand_pos == ob.rng_state().libc_rand_pos
    ga.close()
    gb.close()


def test_process_statics_one_sharded_context_per_process(gpu_mod):
    """ESLAM_FLAG_PROCESS_STATICS with ranks in one process: two rank contexts would share the
    respawn counter and rand() and their collectives would diverge, so eslam_gpu_set_comm
    refuses the second one (ESLAM_ERR_INVALID_ARG); returning the first context to one GPU
    (comm == NULL) frees the place.  set_comm itself runs no exchange, so the callbacks here
    are never called."""
    import ctypes as C
    import eslam_abi as A
    n = 4096
    cfg = hash_config(n, steps=4, bins=20, period=3)
    cfg.flags |= A.FLAG_PROCESS_STATICS

    def never(*args):
        raise AssertionError("set_comm ran a collective")
    ag, a2a = A.ALLGATHER_FN(never), A.ALLTOALLV_FN(never)
    bounds = A.shard_bounds(n, 2)
    gb = (C.c_uint64 * len(bounds))(*bounds)
    fa, fb = gpu_mod.GpuFilter(cfg), gpu_mod.GpuFilter(cfg)
    ca, cb = A.Comm(None, 0, 2, 0, 0, ag, a2a), A.Comm(None, 1, 2, 0, 0, ag, a2a)
    assert fa.L.eslam_gpu_set_comm(fa.h, C.byref(ca), n, gb) == 0
    assert fb.L.eslam_gpu_set_comm(fb.h, C.byref(cb), n, gb) == A.ERR_INVALID_ARG
    assert "PROCESS_STATICS" in fb.L.eslam_gpu_last_error(fb.h).decode()
    assert fa.L.eslam_gpu_set_comm(fa.h, None, 0, None) == 0
    assert fb.L.eslam_gpu_set_comm(fb.h, C.byref(cb), n, gb) == 0
    assert fb.L.eslam_gpu_set_comm(fb.h, None, 0, None) == 0
    fa.close()
    fb.close()
