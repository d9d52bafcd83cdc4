"""The oracle built with 288-byte particle records (-DOR_AOS; bench.py's AoS cpu_baseline) gives
the same results as the SoA oracle: against the committed golden vectors, and SoA == AoS bit for
bit in the reference-sum mode the baseline runs in, per-particle maps included."""
import numpy as np
import pytest

from dist_scenarios import run_scenario, scenario_config
from golden_scenarios import SCENARIOS, run
from test_golden import compare


@pytest.mark.parametrize("name", SCENARIOS)
def test_aos_oracle_matches_golden(oracle, name):
    import oracle_ffi as O
    compare(run(name, lambda cfg: O.OracleFilter(cfg, O.SUM_CONTRACT, aos=True), lambda f: f.info()), name)


@pytest.mark.parametrize("name,n", [("forced", 3000), ("natural", 2000), ("upload", 1500), ("hash", 1200),
                                    ("maps", 600)])
def test_aos_equals_soa_reference_sums(oracle, name, n):
    import oracle_ffi as O
    recs = []
    for aos in (False, True):
        f = O.OracleFilter(scenario_config(name, n), O.SUM_REFERENCE, aos=aos)
        recs.append(run_scenario(f, name, n, 0, n, info_fn=lambda g: g.info()))
    soa, aos = recs
    assert set(soa) == set(aos)
    for k in soa:
        a, b = np.ascontiguousarray(soa[k]), np.ascontiguousarray(aos[k])
        assert a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8)), k
