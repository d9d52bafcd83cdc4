#!/bin/bash
# PMC passes of the per-particle map update (bench.py --local-maps), one rocprofv3 run per
# pass: instruction mix and wave states, then memory (L2 hits, TLB translation misses).
# Usage (GPU box): bash tools/pmc_maps.sh <tag> [bench args...]
cd "$(dirname "$0")/.."
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1 || true
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
            "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu-baseline --local-maps "$@" > $out/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $out/p$i.log; }
done
python3 - "$out" <<'PY'
import csv, glob, os, sys, json
from collections import defaultdict
d = sys.argv[1]
res = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("eslam_dev::", "")
        res[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in res.items()}
json.dump(out, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
for k, cs in out.items():
    if "map" in k or "project" in k:
        print(k, json.dumps({c: round(v) for c, v in sorted(cs.items())}))
PY
