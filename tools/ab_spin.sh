#!/bin/bash
# A/B of the sharded step's host spin bound (ESLAM_SPIN_US) on one rank, interleaved.
# Usage (GPU box): bash tools/ab_spin.sh
cd "$(dirname "$0")/.."
out=gpurun_out/ab_spin.log
mkdir -p gpurun_out
: > $out
for rep in 1 2 3; do
  for n in 4194304 2097152; do
    for us in 200 2000; do
      line=$(ESLAM_SPIN_US=$us timeout -k 10 120 python bench.py --sharded --particles $n --steps 50 --warmup 10 --no-cpu-baseline 2>/dev/null) || { echo "FAIL us=$us n=$n" >> $out; exit 1; }
      echo "rep=$rep n=$n spin_us=$us $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out
    done
  done
done
cat $out
