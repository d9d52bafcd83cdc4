#!/bin/bash
# Interleaved A/B of library builds on one GPU box, with one SQ instruction-count pass per
# library:  bash tools/ab_libs.sh <tag> <reps> "<particle counts>" lib1.so lib2.so ...
# (PMC="<counters>" replaces the SQ instruction counters; BENCH_ARGS adds bench.py flags)
# Output: gpurun_out/<tag>/ab.log (value, ms/step, kernel ms per run) and pmc_<lib>.csv.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; reps=$2; sizes=$3; shift 3
out=gpurun_out/$tag
mkdir -p $out
for n in $sizes; do
  for r in $(seq 1 $reps); do
    for lib in "$@"; do
      printf "n=%s %s " $n "$(basename $lib)" | tee -a $out/ab.log
      ESLAM_GPU_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --particles $n $BENCH_ARGS \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])" | tee -a $out/ab.log
      [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
    done
  done
done
for lib in "$@"; do
  b=$(basename $lib .so)
  ESLAM_GPU_LIB=$PWD/$lib timeout -s KILL 90 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU} \
    --output-format csv -d $out/pmc_$b -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > $out/pmc_$b.log 2>&1 || { echo "pmc $b failed"; exit 1; }
done
python3 - "$out" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    res = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("eslam_dev::", "")
        res[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("==", f.split(os.sep)[2])
    for k, cs in res.items():
        if "project_weight" in k or "normalize" in k or "map_merge" in k:
            print(" ", k[:60], {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
