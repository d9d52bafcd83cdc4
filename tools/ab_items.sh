#!/bin/bash
# fused K3 tile size A/B (interleaved): bash tools/ab_items.sh "<particle counts>" "<items list>"
cd "$(dirname "$0")/.."
for n in $1; do
  for r in 1 2 3; do
    for it in $2; do
      printf "n=%s items=%s " $n $it
      ESLAM_SCAN_ITEMS=$it timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --particles $n | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'])" || exit 1
    done
  done
done
