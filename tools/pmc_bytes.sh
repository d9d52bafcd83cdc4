#!/bin/bash
# HBM bytes per kernel dispatch (separate FETCH_SIZE and WRITE_SIZE passes; gfx950: FETCH_SIZE
# x2 for wide coalesced reads, MI355X_MICROARCH.md) of bench.py with the given arguments.
# Usage (GPU box): bash tools/pmc_bytes.sh <tag> [bench args...]
cd "$(dirname "$0")/.."
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmcb_$tag
mkdir -p $out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $out/$c -o run -- python3 bench.py --no-cpu-baseline "$@" > $out/$c.log 2>&1 || { echo "$c rc=$?"; tail -3 $out/$c.log; exit 1; }
done
python3 - "$out" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, c, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == c:
                acc[row["Kernel_Name"].split("(")[0].replace("void ", "").replace("eslam_dev::", "")].append(float(row["Counter_Value"]))
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]) / len(kv[1]))[:8]:
        print(f"{c:10s} {k[:50]:50s} calls {len(v):4d} avg {sum(v) / len(v) / 1024:10.1f} MiB (raw KiB units)")
PY
