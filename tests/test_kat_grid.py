"""The reference's contact-model KATs (test/testContactModel.cpp) through the whole filter: a
one-particle oracle filter on the 2 x 2-cell grid that reproduces FakeMLSAccess
(tests/kat_grid.py) runs updateWeights, and the contact model's outputs it captured (found
points, getWeight / getZDelta / getZVar) meet the reference's expected values.  The same inputs
go through the HIP library in tests/test_gpu_kats.py, bit for bit against this oracle, which
ties the GPU path to the reference's own known answers."""
import numpy as np
import pytest

import oracle_ffi as O
from kat_grid import CASES, kat_setup


def run_oracle_case(name, literal=False):
    cfg, grid, st, pa, expected = kat_setup(name)
    f = O.OracleFilter(cfg, O.SUM_CONTRACT)
    f.set_literal(literal)
    f.set_debug(True)
    f.set_map(grid)
    f.upload(pa)
    assert f.update(st) == 0
    return f, expected


@pytest.mark.parametrize("literal", [False, True])
@pytest.mark.parametrize("name", sorted(CASES))
def test_kat_through_filter(oracle, name, literal):
    f, exp = run_oracle_case(name, literal)
    ncp, cp, zdelta, zvar = f.debug()
    after = f.download()
    assert int(ncp[0]) == exp["ncp"]
    assert int(after.n_contact_points[0]) == exp["ncp"]
    assert int(after.floating[0]) == (0 if exp["accepted"] else 1)
    if exp["accepted"]:
        # mprob = ContactModel::getWeight() (src/PoseEstimator.cpp:299-301)
        if "weight" in exp:
            assert after.mprob[0] == pytest.approx(exp["weight"], rel=1e-8)      # BOOST_CHECK_CLOSE 1e-6 %
        if "zdelta" in exp:
            assert zdelta[0] == pytest.approx(exp["zdelta"], abs=1e-6)           # BOOST_CHECK_SMALL 1e-6
        if "zvar" in exp:
            rel = 1e-8 if exp["zvar"] < 1e3 else 0.01
            assert zvar[0] == pytest.approx(exp["zvar"], rel=rel)
    else:
        assert after.mprob[0] == 1.0
