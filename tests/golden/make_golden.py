#!/usr/bin/env python3
"""Generate the golden vectors of tests/golden/ from the CPU oracle (contract sums).

    python tests/golden/make_golden.py

Each scenario is a small run (512 particles, 4 steps) of the hot path: the inputs are
regenerated from the scenario parameters (maps, step streams, config - all deterministic,
slam-eslam_amd/synthetic.py), the outputs are every particle field after init and after
every step, the update info, the resample ancestors and the RNG state.  tests/test_golden.py
re-runs the oracle (CPU) and the GPU path (gpu marker) against these files, so a change of
either that alters a result shows up even when both change together.  The reference itself
cannot be built here; its own known-answer tests are in
tests/test_oracle_kats.py.  Regenerate only for a deliberate contract change.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "slam-eslam_amd"))

from golden_scenarios import SCENARIOS, run  # noqa: E402


def main():
    import oracle_ffi as O
    O.build()
    for name in SCENARIOS:
        rec = run(name, lambda cfg: O.OracleFilter(cfg, O.SUM_CONTRACT), lambda f: f.info())
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **rec)
        print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
