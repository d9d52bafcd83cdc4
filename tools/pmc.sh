#!/bin/bash
# Instruction-mix PMC passes (SQ counters) of bench.py, one rocprofv3 run per pass.
# Usage (GPU box): bash tools/pmc.sh <tag> [bench args...]
cd "$(dirname "$0")/.."
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/pmc_$tag
mkdir -p $out
timeout -k 10 120 rocprofv3 -L > $out/counters.txt 2>&1 || true
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
            "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $out/p$i -o run -- python3 bench.py --no-cpu-baseline "$@" > $out/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 $out/p$i.log; }
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
    if k.startswith("k_"):
        print(k, json.dumps({c: round(v) for c, v in sorted(cs.items())}))
PY
