"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same seeded
inputs.  Bit-exact on every particle field, the update info and the resample ancestors."""
import math

import numpy as np
import pytest

import eslam_abi as A
import oracle_ffi as O
import synthetic as S
from parity_util import assert_bit_identical, info_tuple, run_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def flat_grid():
    return S.flat_map(cells=200)


@pytest.fixture(scope="module")
def rough_grid():
    return S.rough_map(cells=200)


def factory(gpu_mod):
    return lambda cfg: gpu_mod.GpuFilter(cfg)


@pytest.mark.parametrize("fn,lo,hi", [(0, -740, 700), (1, 1e-300, 1e300), (2, -50, 50), (3, -50, 50), (4, -8, 27),
                                      (5, 0, 1e10), (8, 0, 1.5), (9, 0, 1.9), (13, 0, 1), (14, 0, 1),
                                      (15, 2.0 ** -33, 1.0), (16, 0, 2.0 ** 32), (17, 0, 2.0 ** 32),
                                      (18, 0, 2.0 ** 32), (19, 0, 2.0 ** 32), (26, 0, 2.0 ** 32), (27, 0, 2.0 ** 32)])
def test_gpu_math_bit_identical(gpu_mod, oracle, fn, lo, hi):
    rng = np.random.default_rng(fn)
    x = rng.uniform(lo, hi, 20000) if fn != 1 else np.exp(rng.uniform(-690, 690, 20000))
    y = rng.uniform(0, 4, 20000)
    if fn >= 16:                          # 32-bit words
        x = np.floor(x)
        y = np.floor(rng.uniform(0, 2.0 ** 32, 20000))
    if fn == 8:
        y = np.where(rng.random(20000) < 0.5, np.floor(y), 1.0 / rng.integers(1, 9, 20000))
    got = gpu_mod.selftest_math(fn, x, y)
    want = np.array([oracle.dm(fn, float(a), float(b)) for a, b in zip(x, y)])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), f"fn {fn}: {np.count_nonzero(got != want)} differ"


def test_box_muller_radius_all_words(gpu_mod):
    """dm_sqrtf_pos(x) == sqrtf(x), x = (float)(-2 dm_log_bm(u)), bit for bit on the device for
    every one of the 2^32 uniform words: the range-restricted fp32 sqrt of the Box-Muller
    radius is correctly rounded there (the oracle uses the C library's sqrtf)."""
    import ctypes as C
    L = gpu_mod.load_library()
    bad = C.c_uint64(1)
    assert L.eslam_gpu_selftest_bm_radius(0, C.byref(bad)) == 0
    assert bad.value == 0


def test_lane_exchange(gpu_mod):
    """The DPP / permlane lane exchanges behind every wave butterfly (the sum contract's chunk
    tree): lane i receives exactly lane i ^ 2^k's 64-bit value, k = 0..5."""
    rng = np.random.default_rng(11)
    x = rng.standard_normal(1024)
    idx = np.arange(x.size)
    for k in range(6):
        got = gpu_mod.selftest_math(20 + k, x)
        assert np.array_equal(got.view(np.uint64), x[idx ^ (1 << k)].view(np.uint64)), f"xor {1 << k}"


def test_gpu_div_and_ratio(gpu_mod, oracle):
    rng = np.random.default_rng(7)
    x = rng.normal(size=20000) * 10.0 ** rng.uniform(-5, 5, 20000)
    y = 10.0 ** rng.uniform(-3, 3, 20000)
    for fn in (6, 7):
        got = gpu_mod.selftest_math(fn, x, y)
        want = np.array([oracle.dm(fn, float(a), float(b)) for a, b in zip(x, y)])
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_flat_forced_resample(gpu_mod, flat_grid):
    cfg = S.bench_config(A.default_config(), 1000)
    run_pair(cfg, flat_grid, S.step_stream(8), 1000, gpu_factory=factory(gpu_mod), label="flat")


def test_rough_tilted_natural_gate(gpu_mod, rough_grid):
    cfg = A.default_config()
    cfg.particle_count = 3000
    run_pair(cfg, rough_grid, S.step_stream(25, tilt=True), 3000, gpu_factory=factory(gpu_mod), label="rough")


def test_rough_forced_every_step_ragged(gpu_mod, rough_grid):
    n = 4097                       # not a multiple of 64 or of the 2048-particle scan tile
    cfg = S.bench_config(A.default_config(), n)
    run_pair(cfg, rough_grid, S.step_stream(6, tilt=True), n, gpu_factory=factory(gpu_mod), label="ragged")


def test_two_item_scan_band(gpu_mod, rough_grid):
    """n in (2^18, 2^19]: the 2-items-per-thread instantiation of k_normalize_segments
    (eslam_ctx.hip scan_items), with a ragged last tile; every particle after every step."""
    n = 400003
    cfg = S.bench_config(A.default_config(), n)
    run_pair(cfg, rough_grid, S.step_stream(3, tilt=True), n, gpu_factory=factory(gpu_mod), label="400k")


def test_grouped_nan_contacts_and_misses(gpu_mod, rough_grid):
    # 8 contacts in 4 groups of 2 (asguard-like wheels), NaN = unknown contact probability
    feet = [(0.3, 0.1, -0.18), (0.3, -0.1, -0.2), (-0.3, 0.1, -0.18), (-0.3, -0.1, -0.22),
            (0.3, -0.5, -0.18), (0.3, -0.7, -0.19), (-0.3, -0.5, -0.18), (-0.3, -0.7, -0.25)]
    groups = [0, 0, 1, 1, 2, 2, 3, 3]
    contact = lambda s, i: float("nan") if (s + i) % 3 == 0 else (0.1 if (s * 7 + i) % 5 == 0 else 0.9)
    stream = S.step_stream(10, tilt=True, feet=feet, groups=groups, contact=contact, ltc=1)
    cfg = A.default_config()
    cfg.particle_count = 2000
    cfg.min_contacts = 2
    run_pair(cfg, rough_grid, stream, 2000, init=dict(mu=[0, 0, 0], sigma=[3.0, 3.0, 1.0], z=0.18, zs=0.3),
             gpu_factory=factory(gpu_mod), label="grouped")


def test_particles_leaving_the_map(gpu_mod):
    grid = S.flat_map(cells=20)    # 2 x 2 m map: most feet miss (GridAccess::get false)
    cfg = S.bench_config(A.default_config(), 1500)
    run_pair(cfg, grid, S.step_stream(6), 1500, init=dict(mu=[0.5, 0.5, 0], sigma=[1.5, 1.5, 0.5], z=0.18, zs=0.5),
             gpu_factory=factory(gpu_mod), label="offmap")


def test_all_floating_uniform_reset(gpu_mod):
    grid = S.flat_map(cells=20)
    cfg = A.default_config()
    cfg.particle_count = 700
    # every particle far away from the map: no contact points, data_particles == 0;
    # initial weights are 0 (Q3) so normalizeWeights takes the uniform branch
    run_pair(cfg, grid, S.step_stream(4, ltc=1), 700, init=dict(mu=[40, 40, 0], sigma=[0.1, 0.1, 0.1], z=0.18, zs=1.0),
             gpu_factory=factory(gpu_mod), label="uniform")


def test_uploaded_large_weights(gpu_mod, rough_grid):
    n = 2500
    rng = np.random.default_rng(5)
    pa = A.ParticleArrays(n)
    pa.x[:] = rng.normal(0, 0.2, n)
    pa.y[:] = rng.normal(0, 0.2, n)
    pa.orientation[:] = rng.normal(0, 0.1, n)
    pa.zpos[:] = 0.18
    pa.zsigma[:] = 0.2
    pa.weight[:] = rng.uniform(0, 37.5, n)      # unnormalised, > 1: exercises the weight exponent
    pa.floating[:] = 1
    cfg = S.bench_config(A.default_config(), n)
    run_pair(cfg, rough_grid, S.step_stream(5, tilt=True), n, init=pa, gpu_factory=factory(gpu_mod), label="upload")


def test_project_then_update_separately(gpu_mod, flat_grid):
    cfg = S.bench_config(A.default_config(), 1200)
    stream = S.step_stream(4)
    gpu, orc = run_pair(cfg, flat_grid, stream, 1200, gpu_factory=factory(gpu_mod), mode="project", label="project")
    for k, st in enumerate(stream):
        orc.update(st)
        gpu.update(st)
        gpu.sync()
        assert_bit_identical(gpu.download(), orc.download(), f"update {k}")
        assert info_tuple(gpu.sync()) == info_tuple(orc.info())


def test_particle_filter_api(gpu_mod, rough_grid):
    """getWeightsSum, normalizeWeights, resample (unnormalised weights), getBestParticleIndex,
    getCentroid (src/ParticleFilter.hpp:34-173, src/PoseEstimator.cpp:354-383)."""
    n = 3333
    rng = np.random.default_rng(11)
    pa = A.ParticleArrays(n)
    pa.x[:] = rng.normal(0, 1, n)
    pa.y[:] = rng.normal(0, 1, n)
    pa.orientation[:] = rng.normal(0, 0.3, n)
    pa.zpos[:] = rng.normal(0.2, 0.01, n)
    pa.zsigma[:] = 0.1
    pa.weight[:] = np.exp(-0.5 * (pa.x ** 2 + pa.y ** 2)) / math.sqrt(2 * math.pi)   # like UnitTest.cpp's tracker
    pa.weight[17] = pa.weight.max()                                                   # tie: first max wins
    cfg = A.default_config()
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    orc = O.OracleFilter(cfg)
    gpu = gpu_mod.GpuFilter(cfg)
    orc.upload(pa)
    gpu.upload(pa)
    assert gpu.weights_sum() == orc.weights_sum()
    assert gpu.best_index() == orc.best_index()
    gpu.resample()
    orc.resample()
    gpu.sync()
    assert np.array_equal(gpu.ancestors(), orc.ancestors())
    assert_bit_identical(gpu.download(), orc.download(), "resample")
    assert gpu.normalize() == orc.normalize()
    assert_bit_identical(gpu.download(), orc.download(), "normalize")
    assert gpu.count() == n
    # getCentroid: the device sums in the canonical chunk order + a fixed tree, as the
    # contract oracle does (bit for bit); the reference's sequential sums agree to 1e-12
    ref = O.OracleFilter(cfg, O.SUM_REFERENCE)
    ref.upload(orc.download())
    gp, gq = gpu.centroid()
    op, oq = orc.centroid()
    rp, rq = ref.centroid()
    assert np.array_equal(np.array(gp + gq).view(np.uint64), np.array(op + oq).view(np.uint64)), (gp, op)
    assert np.allclose(gp, rp, rtol=1e-12, atol=1e-15), (gp, rp)
    assert np.allclose(gq, rq, rtol=1e-12, atol=1e-15), (gq, rq)


def test_rng_state_resume(gpu_mod, flat_grid):
    cfg = S.bench_config(A.default_config(), 1000)
    stream = S.step_stream(6)
    a = gpu_mod.GpuFilter(cfg)
    a.set_map(flat_grid)
    a.init_gaussian(1000, [0, 0, 0], [0.1, 0.1, 0.1], 0.18, 1.001)
    for st in stream[:3]:
        a.step(st)
    a.sync()
    snap = a.download()
    rs = a.rng_state()
    for st in stream[3:]:
        a.step(st)
    a.sync()
    b = gpu_mod.GpuFilter(cfg)
    b.set_map(flat_grid)
    b.upload(snap)
    b.set_rng_state(rs)
    # upload re-derives the weight exponent; the snapshot weights are normalised (exp 1)
    for st in stream[3:]:
        b.step(st)
    b.sync()
    assert_bit_identical(b.download(), a.download(), "resume")


@pytest.mark.parametrize("profile", ["chunks", "heavy", "single"])
def test_resample_concentrated_weights(gpu_mod, profile):
    """Stratified resample where one wave's particles receive far more than 512 draws: two LDS
    chunks of draws (profile "chunks"), the per-target window path ("heavy"), one particle with
    all the weight ("single").  Ancestors and particles bit-exact against the oracle."""
    n = 20000
    rng = np.random.default_rng(23)
    pa = A.ParticleArrays(n)
    pa.x[:] = rng.normal(0, 0.2, n)
    pa.y[:] = rng.normal(0, 0.2, n)
    pa.orientation[:] = rng.normal(0, 0.1, n)
    pa.zpos[:] = 0.18
    pa.zsigma[:] = 0.2
    w = rng.uniform(0.5, 1.5, n)
    if profile == "chunks":
        w[4096:6144] *= 1.7              # ~1.7x the draws of an average wave over four waves
    elif profile == "heavy":
        w[5000] = 4000.0                 # ~17 % of all draws on one particle
        w[12000:12010] = 300.0
    else:
        w[:] = 0.0
        w[7777] = 0.25
    pa.weight[:] = w
    cfg = A.default_config()
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    orc = O.OracleFilter(cfg)
    gpu = gpu_mod.GpuFilter(cfg)
    orc.upload(pa)
    gpu.upload(pa)
    gpu.resample()
    orc.resample()
    gpu.sync()
    assert np.array_equal(gpu.ancestors(), orc.ancestors())
    assert_bit_identical(gpu.download(), orc.download(), "resample " + profile)


def test_resample_window_bounds_low_half_bit31(gpu_mod):
    """K3b keeps each wave's cumulative-sum range [wlo, whi] in SGPRs (readfirstlane of the two
    32-bit halves).  A build once widened the low half with sign extension, which turned every
    bound whose low half has bit 31 set into 0xffffffff in the high word and faulted the GPU
    (DESIGN.md 4).  Here every wave boundary of the only tile has exactly that low half:
    weights 1.0 except w[0] = 1 + 2^-17, so at the resample's fixed-point shift of 48 (sum 2048:
    61 - (12 + 1)) the prefix at 512 k is (512 k) 2^48 + 2^31.  Ancestors bit-exact vs the oracle
    (src/ParticleFilter.hpp:85-108)."""
    n = 2048
    pa = A.ParticleArrays(n)
    pa.x[:] = np.arange(n) * 1e-3
    pa.zpos[:] = 0.18
    pa.zsigma[:] = 0.2
    pa.weight[:] = 1.0
    pa.weight[0] = 1.0 + 2.0 ** -17
    shift = 61 - (12 + 1)
    for k in (1, 2, 3):
        fx = (512 * k) * 2 ** shift + 2 ** 31        # exact prefix at the wave boundary
        assert (fx & 0xffffffff) >> 31 == 1 and fx >> 32 != 0
    cfg = A.default_config()
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    orc = O.OracleFilter(cfg)
    gpu = gpu_mod.GpuFilter(cfg)
    orc.upload(pa)
    gpu.upload(pa)
    gpu.resample()
    orc.resample()
    gpu.sync()
    anc = gpu.ancestors()
    assert np.array_equal(anc, orc.ancestors())
    assert_bit_identical(gpu.download(), orc.download(), "bit31 bounds")


def test_zero_measurement_variance_stops_the_update(gpu_mod, oracle):
    """measurementError = 0 and zSigma = 0 make measVar = 0: evaluatePose throws
    (src/ContactModel.cpp:122-123) from inside updateWeights' particle loop.  The step reports
    ESLAM_ERR_ZERO_MEAS_VAR from the call itself; phase A has run on every particle, phase B,
    normalizeWeights and resample have not, and the update gate pose is not advanced
    (src/EmbodiedSlamFilter.cpp:361-362) -- so the gate fires again on the next step.  Natural
    gate thresholds; the oracle returns the same code from or_step.  Bit-exact after every step."""
    import ctypes as C
    n = 1000
    grid = S.flat_map(cells=200)
    cfg = A.default_config()
    cfg.particle_count = n
    cfg.measurement_error = 0.0
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    stream = S.step_stream(14)
    for st in stream:
        st.position_error_zz = 0.0                  # project keeps zSigma = 0
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 0.0)
    errors = 0
    for k, st in enumerate(stream):
        u = C.c_int(0)
        orc_rc = orc.L.or_step(orc.h, C.byref(st), C.byref(u))
        try:
            gpu.step(st)
            gpu_rc = 0
        except gpu_mod.EslamError as e:
            gpu_rc = e.code
        assert gpu_rc == orc_rc, (k, gpu_rc, orc_rc)
        errors += gpu_rc == A.ERR_ZERO_MEAS_VAR
        gpu.sync()
        assert_bit_identical(gpu.download(), orc.download(), f"zero-var step {k}")
        assert info_tuple(gpu.sync()) == info_tuple(orc.info()), k
    assert errors >= 2                              # the gate fired again after the first throw


@pytest.mark.parametrize("case", ["nan_in_window", "far_and_inf"])
def test_nonfinite_and_off_grid_particles(gpu_mod, rough_grid, case):
    """Particles with NaN, infinite, far-off and grid-edge coordinates take the map lookup's
    window test and its global fallback exactly as the oracle's getPatch: NaN coordinates
    inside a staged LDS window (the cloud's box skips them), and off-grid values that clamp
    in the cell conversion with the window off."""
    n = 4096
    rng = np.random.default_rng(5)
    pa = A.ParticleArrays(n)
    pa.x[:] = rng.normal(0.0, 0.1, n)
    pa.y[:] = rng.normal(0.0, 0.1, n)
    pa.orientation[:] = rng.normal(0.0, 0.05, n)
    pa.zpos[:] = 0.18
    pa.zsigma[:] = 0.5
    pa.weight[:] = 1.0
    pa.mprob[:] = 1.0
    pa.floating[:] = 1
    pa.n_contact_points[:] = 0
    idx = rng.choice(n, 300, replace=False)
    if case == "nan_in_window":
        pa.x[idx[:100]] = math.nan
        pa.y[idx[100:200]] = math.nan
        pa.x[idx[200:]] = math.nan
        pa.y[idx[200:]] = math.nan
    else:
        vals = np.array([math.inf, -math.inf, 1e12, -1e12, -10.05, 10.05, 9.999, -9.999, 3e9, -3e9])
        pa.x[idx[:150]] = rng.choice(vals, 150)
        pa.y[idx[150:]] = rng.choice(vals, 150)
    cfg = S.bench_config(A.default_config(), n)
    run_pair(cfg, rough_grid, S.step_stream(4), n, init=pa, gpu_factory=factory(gpu_mod), label=case)
