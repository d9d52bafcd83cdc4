#!/usr/bin/env python3
"""Probe (GPU box): two ranks of the library's own RCCL communicator (eslam_gpu_set_comm_rccl)
on ONE GPU, the 'forced' scenario at 5000 particles, against the one-process CPU oracle bit
for bit.  RCCL normally refuses two ranks on one device; this records what it does here.

    timeout -k 10 150 python tools/rccl_two_ranks_probe.py <out_dir>
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

import conftest  # noqa: F401,E402  (sys.path for the package and the oracle)
from test_dist_cpu import assert_same, launch, merge, single_oracle  # noqa: E402


def main(out):
    import oracle_ffi
    oracle_ffi.build()
    os.makedirs(out, exist_ok=True)
    want = single_oracle("forced", 5000)
    parts = launch("gpu", "forced", 5000, 2, out, mem="rccl", timeout=120)
    assert_same(merge(parts), want, "gpu native rccl forced N=5000 world=2 (one GPU)")
    print("rccl two ranks on one GPU: sharded == single oracle, bit for bit")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rccl2")
