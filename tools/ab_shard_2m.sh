#!/bin/bash
# configs[3]'s per-GPU size (2M particles): single-GPU path vs the sharded path on one rank,
# interleaved.  Usage (GPU box): bash tools/ab_shard_2m.sh
cd "$(dirname "$0")/.."
out=gpurun_out/ab_shard_2m.log
mkdir -p gpurun_out
: > $out
for rep in 1 2 3; do
  for mode in single sharded; do
    flag=""; [ $mode = sharded ] && flag="--sharded"
    line=$(timeout -k 10 120 python bench.py $flag --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline 2>/dev/null) || { echo "FAIL $mode" >> $out; exit 1; }
    echo "rep=$rep n=2097152 $mode $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernel_ms"]; print(d["value"], d["ms_per_step"], json.dumps(k))')" >> $out
  done
done
cat $out
