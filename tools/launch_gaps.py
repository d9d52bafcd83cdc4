#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps between consecutive dispatches of a rocprofv3
kernel trace (run_kernel_trace.csv): python tools/launch_gaps.py <trace dir> [last N dispatches]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rows = rows[-last:]
dur = defaultdict(list)
gap_before = defaultdict(list)
for prev, cur in zip(rows, rows[1:]):
    name = cur["Kernel_Name"].split("(")[0]
    dur[name].append((int(cur["End_Timestamp"]) - int(cur["Start_Timestamp"])) / 1e3)
    gap_before[name].append((int(cur["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
busy = sum(sum(v) for v in dur.values())
print(f"{len(rows)} dispatches, span {span:.1f} us, kernels busy {busy:.1f} us ({100 * busy / span:.1f} %)")
for k in dur:
    print(f"{k:60s} n={len(dur[k]):4d} median {statistics.median(dur[k]):7.2f} us, "
          f"gap before it: median {statistics.median(gap_before[k]):5.2f} us, max {max(gap_before[k]):6.2f} us")
