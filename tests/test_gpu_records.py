"""PoseParticle records with the debug fields (eslam_gpu_download_records): the cpoints,
meas_pos and meas_theta updateWeights stores in every particle (src/PoseEstimator.cpp:285-287,
322-325; ContactPoint src/PoseParticle.hpp:20-43, filled at src/ContactModel.cpp:163-207),
carried through the resample with the particle, as the viz reads them
(viz/ParticleVisualization.cpp:111-213).  Bit-exact against the oracle's per-particle
capture (or_set_debug), mapped through the oracle's ancestors."""
import numpy as np
import pytest

import eslam_abi as A
import golden_scenarios as G
import oracle_ffi as O
import synthetic as S
from parity_util import assert_bit_identical

pytestmark = pytest.mark.gpu
MAXC = 8


def u64(a):
    return np.ascontiguousarray(a).view(np.uint64)


def expected_cpoints(orc, n):
    ncp, cp, _, _ = orc.debug()
    info = orc.info()
    anc = orc.ancestors().astype(np.int64) if info.resampled else np.arange(n)
    raw = np.ctypeslib.as_array(cp).reshape(n, A.MAX_CONTACTS)
    return ncp[anc], raw[anc]


@pytest.mark.parametrize("name", ["grouped_nan", "rough_natural", "flat_forced"])
def test_records_match_oracle_capture(gpu_mod, oracle, name):
    cfg, grid, stream, init = G.setup(name)
    cfg.flags |= A.FLAG_RECORD_CONTACTS
    n = cfg.particle_count
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_debug(True)
    for f in (gpu, orc):
        f.set_map(grid)
        f.init_gaussian(n, init["mu"], init["sigma"], init["z"], init["zs"])
    updates = 0
    for k, st in enumerate(stream):
        assert gpu.step(st) == orc.step(st)
        gpu.sync()
        assert_bit_identical(gpu.download(), orc.download(), f"{name} step {k}")
        if orc.info().update_count == 0:
            continue
        updates += 1
        rec, cps = gpu.download_records(max_cpoints=MAXC)
        want_n, want_cp = expected_cpoints(orc, n)
        assert np.array_equal(rec["n_cpoints"], want_n), f"{name} step {k}: cpoints.size()"
        for q in range(MAXC):
            has = want_n > q
            g, w = cps[has, q], want_cp[has, q]
            for fld in ("zdiff", "zvar", "prob"):
                assert np.array_equal(u64(g[fld]), u64(w[fld])), (name, k, q, fld)
            assert np.array_equal(u64(g["point"]), u64(w["point"])), (name, k, q, "point")
        p = gpu.download()
        assert np.array_equal(u64(rec["position"][:, 0]), u64(p.x))
        assert np.array_equal(u64(rec["meas_pos"][:, 0]), u64(p.x)), "meas_pos.x = x at the update"
        assert np.array_equal(u64(rec["meas_pos"][:, 1]), u64(p.y))
        assert np.array_equal(u64(rec["meas_theta"]), u64(p.orientation))
        assert np.array_equal(rec["index"], np.arange(n))
    assert updates >= 2


def test_records_strided_without_capture(gpu_mod):
    """Without the capture flag the records are the particle fields (a strided device-side
    gather, one copy), n_cpoints the last update's count and meas_* zero."""
    n = 5000
    cfg = S.bench_config(A.default_config(), n)
    gpu = gpu_mod.GpuFilter(cfg)
    gpu.set_map(S.flat_map(cells=200))
    gpu.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    for st in S.step_stream(3):
        gpu.step(st)
    rec, cps = gpu.download_records(first=3, stride=7)
    assert cps is None
    p = gpu.download()
    idx = np.arange(3, n, 7)
    assert len(rec) == idx.size and np.array_equal(rec["index"], idx)
    for fld, col in (("orientation", p.orientation), ("zpos", p.zpos), ("zsigma", p.zsigma), ("weight", p.weight),
                     ("mprob", p.mprob)):
        assert np.array_equal(u64(rec[fld]), u64(col[idx])), fld
    assert np.array_equal(rec["n_cpoints"], p.n_contact_points[idx].astype(np.uint32))
    assert np.array_equal(rec["floating"], p.floating[idx])
    assert not rec["meas_pos"].any()
    with pytest.raises(gpu_mod.EslamError):
        gpu.download_records(first=n - 1, stride=1, count=2)
