"""The committed golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py)
against the CPU oracle and, with the gpu marker, against the GPU path: bit for bit."""
import os

import numpy as np
import pytest

from golden_scenarios import SCENARIOS, run

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def compare(got, name):
    want = dict(np.load(os.path.join(GOLDEN, f"{name}.npz")))
    assert set(got) == set(want), sorted(set(got) ^ set(want))
    for k in want:
        g, w = np.ascontiguousarray(got[k]), np.ascontiguousarray(want[k])
        assert g.shape == w.shape and np.array_equal(g.view(np.uint8), w.view(np.uint8)), \
            f"{name} {k}: {np.count_nonzero(g != w)} entries differ"


@pytest.mark.parametrize("name", SCENARIOS)
def test_oracle_matches_golden(oracle, name):
    import oracle_ffi as O
    compare(run(name, lambda cfg: O.OracleFilter(cfg, O.SUM_CONTRACT), lambda f: f.info()), name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", SCENARIOS)
def test_gpu_matches_golden(name):
    import eslam_amd
    compare(run(name, lambda cfg: eslam_amd.GpuFilter(cfg), lambda f: f.sync()), name)
