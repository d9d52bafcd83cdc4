"""Shared helpers for the GPU-vs-oracle parity tests (test infrastructure)."""
import math
import os
import struct

import numpy as np

import eslam_abi as A
import oracle_ffi as O
import synthetic as S

FLOAT_FIELDS = ("x", "y", "orientation", "zpos", "zsigma", "weight", "mprob")
BYTE_FIELDS = ("floating", "n_contact_points")


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def assert_bit_identical(got, want, label=""):
    """Particle sets equal bit for bit (NaN payloads included)."""
    assert got.n == want.n, f"{label}: count {got.n} != {want.n}"
    for f in FLOAT_FIELDS:
        g, w = bits(getattr(got, f)), bits(getattr(want, f))
        bad = np.nonzero(g != w)[0]
        if bad.size:
            i = int(bad[0])
            gv, wv = getattr(got, f)[i], getattr(want, f)[i]
            raise AssertionError(f"{label}: field {f} differs at {bad.size} particles; first {i}: "
                                 f"gpu {gv!r} oracle {wv!r}")
    for f in BYTE_FIELDS:
        g, w = getattr(got, f), getattr(want, f)
        bad = np.nonzero(g != w)[0]
        if bad.size:
            i = int(bad[0])
            raise AssertionError(f"{label}: field {f} differs at {bad.size} particles; first {i}: gpu {g[i]} oracle {w[i]}")


def assert_close(got, want, rel=1e-6, label=""):
    for f in FLOAT_FIELDS:
        g, w = getattr(got, f), getattr(want, f)
        ok = np.isclose(g, w, rtol=rel, atol=0.0, equal_nan=True)
        assert ok.all(), f"{label}: {f} not within {rel} rel at {np.count_nonzero(~ok)} particles"


def info_tuple(i):
    return (i.effective, i.weight_sum, i.floating_weight, i.max_weight, i.data_particles, i.total_points,
            i.resampled, i.uniform_reset, i.resample_overruns)


def run_pair(cfg, grid, stream, n, init=None, gpu_factory=None, record=True, check_every=True,
             mode="step", label="", oracle_threads=1):
    """Run the same inputs through the oracle (contract sums) and the GPU, comparing after
    every step.  Returns (gpu filter, oracle filter)."""
    if record:
        cfg.flags |= A.FLAG_RECORD_ANCESTORS
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    orc.set_threads(min(oracle_threads, os.cpu_count() or 1))
    gpu = gpu_factory(cfg)
    orc.set_map(grid)
    gpu.set_map(grid)
    if init is None:
        init = dict(mu=[0.0, 0.0, 0.0], sigma=[0.1, 0.1, 0.1], z=0.18, zs=1.001)
    if isinstance(init, A.ParticleArrays):
        orc.upload(init)
        gpu.upload(init)
    else:
        orc.init_gaussian(n, init["mu"], init["sigma"], init["z"], init["zs"])
        gpu.init_gaussian(n, init["mu"], init["sigma"], init["z"], init["zs"])
    assert_bit_identical(gpu.download(), orc.download(), f"{label} init")
    for k, st in enumerate(stream):
        if mode == "step":
            u_o = orc.step(st)
            u_g = gpu.step(st)
            assert u_o == u_g, f"{label} step {k}: update gate differs"
        elif mode == "project":
            orc.project(st)
            gpu.project(st)
            u_o = False
        else:
            orc.update(st)
            gpu.update(st)
            u_o = True
        gi = gpu.sync()
        if check_every or k == len(stream) - 1:
            assert_bit_identical(gpu.download(), orc.download(), f"{label} step {k}")
            if u_o:
                oi = orc.info()
                assert info_tuple(gi) == info_tuple(oi), f"{label} step {k}: info {info_tuple(gi)} != {info_tuple(oi)}"
                if oi.resampled and record:
                    assert np.array_equal(gpu.ancestors(), orc.ancestors()), f"{label} step {k}: ancestors differ"
    return gpu, orc


def check_resample_properties(anc, after, n):
    """Size-independent properties of one stratified resample (src/ParticleFilter.hpp:72-108):
    ancestors nondecreasing and in range; the copies of one ancestor identical in every field
    (the gather copies, Q4: the weights are not reset); each ancestor a copied c_a times with
    |c_a - N w_a| < 2, w_a being its normalised weight (which the copies carry)."""
    anc = np.asarray(anc).astype(np.int64)
    assert anc.shape == (n,)
    assert anc[0] >= 0 and anc[-1] < n and np.all(np.diff(anc) >= 0)
    first = np.r_[True, anc[1:] != anc[:-1]]
    starts = np.nonzero(first)[0]
    copies = np.diff(np.r_[starts, n])
    group = np.cumsum(first) - 1
    for f in FLOAT_FIELDS + BYTE_FIELDS:
        v = getattr(after, f)
        v = v.view(np.uint64) if v.dtype == np.float64 else v
        assert np.array_equal(v, v[starts][group]), f"copies of one ancestor differ in {f}"
    w = after.weight[starts]
    assert np.all(np.abs(copies - n * w) < 2.0)
    assert float(np.sum(w)) <= 1.0 + 1e-9
