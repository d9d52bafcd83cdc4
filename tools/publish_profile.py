#!/usr/bin/env python3
"""Copy a GPU-box profile run (gpurun_out/prof_<tag>, gpurun_out/pmc_<tag>) into the tracked
profiles/<round>/ tree and make it the summary bench.py reads (profiles/<round>/summary.json).

    python tools/publish_profile.py r01 r01e "bash tools/profile.sh r01e --steps 20 --warmup 5" 4194304 1000
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(rnd, tag, command, particles, map_cells):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", rnd, f"prof_{tag}")
    os.makedirs(dst, exist_ok=True)
    summary = json.load(open(os.path.join(src, "summary.json")))
    for f in glob.glob(os.path.join(src, "trace", "*kernel_stats.csv")):
        shutil.copy(f, os.path.join(dst, "kernel_stats.csv"))
    pmc = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}", "pmc_summary.json")
    if os.path.exists(pmc):
        shutil.copy(pmc, os.path.join(dst, "pmc_instruction_mix.json"))
    summary.update(command=command, particles=int(particles), map_cells=int(map_cells))
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1, sort_keys=True)
    json.dump(summary, open(os.path.join(ROOT, "profiles", rnd, "summary.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in summary["kernels"].items() if k.startswith("k_")}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:6])
