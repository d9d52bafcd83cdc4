"""The reference's contact-model KATs (test/testContactModel.cpp:128-362) through the HIP
library: each case is a one-particle update on the 2 x 2-cell FakeMLSAccess grid
(tests/kat_grid.py), run through the C ABI (eslam_gpu_update) and through the CPU oracle.
The GPU's particle and update info equal the oracle's bit for bit, and the quantities the
library exposes meet the reference's expected values: the number of contact points, the
accept / floating decision and mprob = getWeight().  The oracle's getZDelta / getZVar on the
same inputs are checked against the KATs in tests/test_kat_grid.py."""
import pytest

import oracle_ffi as O
from kat_grid import CASES, kat_setup
from parity_util import assert_bit_identical, info_tuple

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_kat(gpu_mod, oracle, name):
    cfg, grid, st, pa, exp = kat_setup(name)
    gpu = gpu_mod.GpuFilter(cfg)
    orc = O.OracleFilter(cfg, O.SUM_CONTRACT)
    for f in (gpu, orc):
        f.set_map(grid)
        f.upload(pa)
    gpu.update(st)
    assert orc.update(st) == 0
    gi = gpu.sync()
    got, want = gpu.download(), orc.download()
    assert_bit_identical(got, want, name)
    assert info_tuple(gi) == info_tuple(orc.info())
    assert int(got.n_contact_points[0]) == exp["ncp"]
    assert int(got.floating[0]) == (0 if exp["accepted"] else 1)
    assert gi.data_particles == (1 if exp["accepted"] else 0)
    if exp["accepted"] and "weight" in exp:
        assert got.mprob[0] == pytest.approx(exp["weight"], rel=1e-8)
