#!/bin/bash
# A/B of library variants at 4M and 256k (interleaved): bash tools/ab_k3.sh lib1.so lib2.so ...
cd "$(dirname "$0")/.."
for n in 4194304 262144; do
  for r in 1 2 3; do
    for lib in "$@"; do
      printf "n=%s %s " $n "$(basename $lib)"
      ESLAM_GPU_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --particles $n | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])" || exit 1
    done
  done
done
