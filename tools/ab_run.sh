#!/bin/bash
# Interleaved A/B timing of alternative library builds: bash tools/ab_run.sh <reps> lib1.so lib2.so ...
cd "$(dirname "$0")/.."
reps=$1; shift
for r in $(seq 1 $reps); do
  for lib in "$@"; do
    printf "%s " "$(basename $lib)"
    ESLAM_GPU_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $BENCH_ARGS | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])" || exit 1
  done
done
