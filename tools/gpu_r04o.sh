#!/bin/bash
# Round 4 final evidence at HEAD: the full GPU suite and smoke, interleaved lines against the
# previous K3 look-back (lib_prev2), the default bench line, kernel trace + PMC passes at 4M,
# the SQ instruction mix, the 256k trace, and the configs[4] lines (bench window and steady
# state).  Stops at a crash or timeout (rc >= 124); test failures are reported and it goes on.
# Usage (GPU box): bash tools/gpu_r04o.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
out=gpurun_out/$tag
mkdir -p $out
L=slam-eslam_amd/lib/ab
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $out/session.log
  [ $rc -lt 124 ] || { tail -30 "$out/$name.log"; exit $rc; }
  return 0
}
line() {  # line <label> <lib or ""> <bench args...>
  local label=$1 lib=$2; shift 2
  printf "%s " "$label" >> $out/lines.log
  if [ -n "$lib" ]; then export ESLAM_GPU_LIB=$PWD/$L/lib_$lib.so; else unset ESLAM_GPU_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $out/tmp.json 2>> $out/bench_err.log || { echo "bench $label failed"; tail -5 $out/bench_err.log; exit 1; }
  unset ESLAM_GPU_LIB
  tail -1 $out/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d.get('kernel_ms')), json.dumps(d.get('map_update', {}).get('patches_covered')))" >> $out/lines.log
}
step pytest_gpu 700 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests
tail -2 $out/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for r in 1 2; do
  for n in 4194304 262144; do
    line "n=$n cur" "" --particles $n --steps 30 --warmup 5
    line "n=$n prev2" prev2 --particles $n --steps 30 --warmup 5
  done
done
cut -c1-220 $out/lines.log
step bench 300 python bench.py
tail -1 $out/bench.log | cut -c1-300
step profile 600 bash tools/profile.sh $tag --steps 50 --warmup 10
step pmc 400 bash tools/pmc.sh $tag --steps 20 --warmup 5
step profile_256k 400 bash tools/profile.sh ${tag}_256k --particles 262144 --steps 50 --warmup 10
line "maps bench window" "" --local-maps --steps 20 --warmup 5
line "maps steady" "" --local-maps --steps 20 --warmup 30
line "sharded 4M" "" --sharded --steps 30 --warmup 5
line "4M" "" --steps 30 --warmup 5
cut -c1-300 $out/lines.log
