"""Parity lineage: the build's arithmetic contract (what the GPU matches bit for bit) against
the reference's literal arithmetic, both on the CPU oracle.

* contract:  OR_SUM_CONTRACT + the contract's formulas (eslam_detmath.h)
* reference: OR_SUM_REFERENCE (the sequential double sums of src/ParticleFilter.hpp:34-108 and
             src/PoseEstimator.cpp:305-310, 329) + or_set_literal (boost's pdf / cdf ratio as libm
             exp / erfc, the divisions of src/ContactModel.cpp:201-203 and 270-301, std::pow,
             libm sin / cos, the fabs / sqrt 1-sigma test)

The same seeded inputs run through both for several forced-resample steps: the resample
ancestors are equal at every step and the weights agree within the north-star tolerance
(1e-6 relative; measured ~1e-12).  Equal ancestors hold on these workloads, not in general: a
stratified draw within rounding of a cumulative-sum boundary could pick the neighbour.  The
random draws (Philox project noise, minstd resample draws) are the build's contract in both
(the reference's boost streams are unpinned).  256k runs in the CPU suite; the
bench's 4M (configs[2]) runs on the GPU box's host cores with the GPU tests."""
import os

import numpy as np
import pytest

import eslam_abi as A
import oracle_ffi as O
import synthetic as S

WEIGHT_TOL = 1e-6          # north-star tolerance on particle weights (BASELINE.json)
REGRESSION_TOL = 1e-9      # what the two arithmetics actually differ by, with margin


def run_lineage(n, terrain, steps, threads):
    cfg = S.bench_config(A.default_config(), n)
    cfg.flags |= A.FLAG_RECORD_ANCESTORS
    grid = S.flat_map(cells=1000) if terrain == "flat" else S.rough_map(cells=1000)
    con = O.OracleFilter(cfg, O.SUM_CONTRACT)
    ref = O.OracleFilter(cfg, O.SUM_REFERENCE)
    ref.set_literal(True)
    worst = {}
    for f in (con, ref):
        f.set_threads(threads)
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    for k, st in enumerate(S.step_stream(steps, tilt=(terrain == "rough"))):
        assert con.step(st) and ref.step(st)
        ci, ri = con.info(), ref.info()
        assert ci.resampled == ri.resampled == 1
        assert np.array_equal(con.ancestors(), ref.ancestors()), f"{terrain} n={n} step {k}: ancestors differ"
        a, b = con.download(), ref.download()
        for fld in ("weight", "x", "y", "orientation", "zpos", "zsigma", "mprob"):
            g, w = getattr(a, fld), getattr(b, fld)
            rel = np.abs(g - w) / np.maximum(np.abs(w), 1e-300)
            worst[fld] = max(worst.get(fld, 0.0), float(rel.max()))
        assert np.array_equal(a.n_contact_points, b.n_contact_points)
        assert np.array_equal(a.floating, b.floating)
        assert ci.effective == pytest.approx(ri.effective, rel=1e-9)
    return worst


def check(worst):
    assert worst["weight"] <= WEIGHT_TOL, worst
    for fld, v in worst.items():
        assert v <= REGRESSION_TOL, (fld, v, worst)


@pytest.mark.parametrize("terrain", ["flat", "rough"])
def test_contract_vs_reference_arithmetic_256k(oracle, terrain):
    check(run_lineage(262144, terrain, 4, os.cpu_count() or 1))


@pytest.mark.gpu              # host-side, but sized for the GPU box's cores and memory
@pytest.mark.timeout(900)
@pytest.mark.parametrize("terrain", ["flat", "rough"])
def test_contract_vs_reference_arithmetic_4m(oracle, terrain):
    check(run_lineage(4 * 1024 * 1024, terrain, 4, min(16, os.cpu_count() or 1)))
