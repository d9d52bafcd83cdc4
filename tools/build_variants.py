"""Experiment builds for interleaved A/B (tools/ab_libs.sh): each variant is a library under
slam-eslam_amd/lib/ab/ built from the current sources with extra defines / flags.
    python tools/build_variants.py name:-DFOO,-DBAR name2:+licm ...
'+licm' drops -disable-machine-licm for the kernels' translation unit."""
import os
import sys
from concurrent.futures import ProcessPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "slam-eslam_amd"))
import build_lib as B  # noqa: E402


def one(spec):
    name, _, opts = spec.partition(":")
    defs = [o[2:] for o in opts.split(",") if o.startswith("-D")]
    out = os.path.join(B.OUT_DIR, "ab")
    os.makedirs(out, exist_ok=True)
    saved = dict(B.PER_SOURCE)
    if "+licm" in opts.split(","):
        B.PER_SOURCE = {}
    try:
        return B.build(force=True, verbose=False, defines=defs, lib=os.path.join(out, f"lib_{name}.so"), tag="_" + name)
    finally:
        B.PER_SOURCE = saved


if __name__ == "__main__":
    with ProcessPoolExecutor(4) as ex:
        for lib in ex.map(one, sys.argv[1:]):
            print(lib)
