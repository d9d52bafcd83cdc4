#!/bin/bash
# Round-4 evidence on one GPU box: rocprofv3 kernel trace + PMC passes of the bench line with
# the in-tree library (profile.sh, pmc.sh), the SQ instruction-mix passes of the round-start
# library for the before/after comparison, and the default bench line.
# Usage (GPU box): bash tools/gpu_r04e.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
out=gpurun_out/$tag
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>: stop at the first failure
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $out/session.log
  [ $rc -eq 0 ] || { tail -30 "$out/$name.log"; exit $rc; }
}
step profile 600 bash tools/profile.sh $tag --steps 50 --warmup 10
step pmc 400 bash tools/pmc.sh $tag --steps 20 --warmup 5
step pmc_base 400 env ESLAM_GPU_LIB=$PWD/slam-eslam_amd/lib/ab/lib_base.so bash tools/pmc.sh ${tag}_base --steps 20 --warmup 5
step bench 300 python bench.py
tail -1 $out/bench.log | cut -c1-600
