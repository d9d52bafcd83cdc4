"""Parity lineage: the build's arithmetic contract (what the GPU matches bit for bit) against
the reference's literal arithmetic, both on the CPU oracle.

* contract:  OR_SUM_CONTRACT + the contract's formulas (eslam_detmath.h)
* reference: OR_SUM_REFERENCE (the sequential double sums of src/ParticleFilter.hpp:34-108 and
             src/PoseEstimator.cpp:305-310, 329) + or_set_literal (boost's pdf / cdf ratio as libm
             exp / erfc, the divisions of src/ContactModel.cpp:201-203 and 270-301, std::pow,
             libm sin / cos, the fabs / sqrt 1-sigma test)

The same seeded inputs run through both for several forced-resample steps.  Each step starts
both filters from the same particles (the contract's state is uploaded into the reference
filter after every step), so every step is compared on its own:

* ancestors: a stratified draw that lies within rounding of a cumulative-sum boundary picks
  the neighbouring particle in one of the two sums.  The reference's sequential double
  cumulative sum (src/ParticleFilter.hpp:95-101) drifts from the exact one by up to ~N eps/4
  (every add rounds at the running total's ulp), and the draws are 1/N apart, so a fraction
  ~N^2 eps of the draws flips: 0-1 over 4 steps at 256k; at 4M (measured over 4 steps, 4 x 4M draws)
  1513 on the flat map (1.2e-4 per draw: identical weights keep the rounding biased) and 38
  on the rough one.  The exact fixed-point sums the GPU uses have no drift.  The test
  asserts that every differing ancestor is an adjacent particle (a boundary flip, not a
  different algorithm) and bounds the flips per step by N^3 2^-53 / 4;
* weights and the other fields of every output whose ancestor agrees: within the north-star
  tolerance (1e-6 relative; measured ~1e-12).

The random draws (Philox project noise, minstd resample draws) are the build's contract in
both (the reference's boost streams are unpinned).  256k runs in the CPU suite; the
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
    worst = {"flips": 0}
    for f in (con, ref):
        f.set_threads(threads)
        f.set_map(grid)
        f.init_gaussian(n, [0.0, 0.0, 0.0], [0.1, 0.1, 0.1], 0.18, 1.001)
    for k, st in enumerate(S.step_stream(steps, tilt=(terrain == "rough"))):
        assert con.step(st) and ref.step(st)
        ci, ri = con.info(), ref.info()
        assert ci.resampled == ri.resampled == 1
        ca, ra = con.ancestors().astype(np.int64), ref.ancestors().astype(np.int64)
        flip = ca != ra
        nflip = int(flip.sum())
        assert np.all(np.abs(ca[flip] - ra[flip]) == 1), f"{terrain} n={n} step {k}: non-adjacent ancestor difference"
        assert nflip <= max(1.0, n * (n * (n * 2.0 ** -53)) / 4), (terrain, n, k, nflip)
        worst["flips"] += nflip
        same = ~flip
        a, b = con.download(), ref.download()
        for fld in ("weight", "x", "y", "orientation", "zpos", "zsigma", "mprob"):
            g, w = getattr(a, fld)[same], getattr(b, fld)[same]
            rel = np.abs(g - w) / np.maximum(np.abs(w), 1e-300)
            worst[fld] = max(worst.get(fld, 0.0), float(rel.max()))
        assert np.array_equal(a.n_contact_points[same], b.n_contact_points[same])
        assert np.array_equal(a.floating[same], b.floating[same])
        assert ci.effective == pytest.approx(ri.effective, rel=1e-9)
        assert con.rng_state().minstd_x == ref.rng_state().minstd_x
        ref.upload(a)                  # the next step starts both from the same particles
    return worst


def check(worst):
    assert worst["weight"] <= WEIGHT_TOL, worst
    for fld, v in worst.items():
        if fld != "flips":
            assert v <= REGRESSION_TOL, (fld, v, worst)


@pytest.mark.parametrize("terrain", ["flat", "rough"])
def test_contract_vs_reference_arithmetic_256k(oracle, terrain):
    check(run_lineage(262144, terrain, 4, os.cpu_count() or 1))


@pytest.mark.gpu              # host-side, but sized for the GPU box's cores and memory
@pytest.mark.timeout(900)
@pytest.mark.parametrize("terrain", ["flat", "rough"])
def test_contract_vs_reference_arithmetic_4m(oracle, terrain):
    check(run_lineage(4 * 1024 * 1024, terrain, 4, min(16, os.cpu_count() or 1)))
