#!/bin/bash
# Interleaved A/B of an environment switch on one library build:
#   bash tools/ab_env.sh <reps> "<particle counts>" VAR=a VAR=b ...
cd "$(dirname "$0")/.."
reps=$1; sizes=$2; shift 2
for n in $sizes; do
  for r in $(seq 1 $reps); do
    for kv in "$@"; do
      printf "n=%s %s " $n "$kv"
      env $kv timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --particles $n $BENCH_ARGS | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'])" || exit 1
    done
  done
done
