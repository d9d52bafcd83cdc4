#!/bin/bash
# interleaved A/B of library builds on the --local-maps bench line (kernel_ms per run):
# bash tools/ab_maps.sh <tag> <reps> lib1.so lib2.so ...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; reps=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for r in $(seq 1 $reps); do
  for lib in "$@"; do
    printf "%s " "$(basename $lib)" | tee -a $out/ab.log
    ESLAM_GPU_LIB=$PWD/$lib timeout -k 10 300 python bench.py --local-maps --steps ${STEPS:-10} --warmup ${WARMUP:-10} --no-cpu-baseline $BENCH_ARGS \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['kernel_ms']; print(d['ms_per_step'], 'merge', round(k['map_merge_ms'],3), 'plan', round(k['map_plan_ms'],3), 'k1', round(k['project_weight_ms'],3))" | tee -a $out/ab.log
    [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
  done
done
