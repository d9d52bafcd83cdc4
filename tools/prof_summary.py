#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel average duration (kernel trace) and HBM
bytes per dispatch from the separate FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE reports half the bytes of coalesced streaming reads -> x2; WRITE_SIZE exact.
    python tools/prof_summary.py gpurun_out/prof_<tag> > summary.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"^void ", "", name)
    n = n.split("(")[0]
    return n.replace("eslam_dev::", "")


def main(d):
    out = {"kernels": {}}
    stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
    if stats:
        for row in csv.DictReader(open(stats[0])):
            out["kernels"].setdefault(short(row["Name"]), {}).update(
                calls=int(row["Calls"]), avg_us=float(row["AverageNs"]) / 1e3, pct=float(row["Percentage"]))
    for counter, sub, corr in (("FETCH_SIZE", "fetch", 2.0), ("WRITE_SIZE", "write", 1.0)):
        files = glob.glob(os.path.join(d, sub, "*counter_collection.csv"))
        if not files:
            continue
        acc = defaultdict(list)
        for row in csv.DictReader(open(files[0])):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
        for k, v in acc.items():
            e = out["kernels"].setdefault(k, {})
            raw = sum(v) / len(v) * 1024.0
            e[counter.lower() + "_raw_bytes"] = raw
            e[counter.lower() + "_bytes"] = raw * corr
    # derived metrics (percent, per dispatch): VALUBusy = SQ_ACTIVE_INST_VALU / CUs / GRBM_GUI_ACTIVE,
    # VALUUtilization = active lanes per VALU instruction
    for counter, sub in (("VALUBusy", "valu"), ("VALUUtilization", "valuutil")):
        files = glob.glob(os.path.join(d, sub, "*counter_collection.csv"))
        if not files:
            continue
        acc = defaultdict(list)
        for row in csv.DictReader(open(files[0])):
            if row["Counter_Name"] == counter:
                acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
        for k, v in acc.items():
            out["kernels"].setdefault(k, {})[counter.lower() + "_pct"] = sum(v) / len(v)
    for k, e in out["kernels"].items():
        if "fetch_size_bytes" in e and "write_size_bytes" in e:
            e["hbm_bytes_per_dispatch"] = e["fetch_size_bytes"] + e["write_size_bytes"]
            if "avg_us" in e:
                e["hbm_gbs"] = e["hbm_bytes_per_dispatch"] / (e["avg_us"] * 1e-6) / 1e9
    out["correction"] = "FETCH_SIZE x2 (gfx950 coalesced-read halving), WRITE_SIZE x1; KiB -> bytes"
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
