#!/bin/bash
# Round-4 evidence: configs[4] A/B of the store-box variants, then the kernel trace + PMC
# passes of the default bench line (in-tree library), the SQ instruction-mix passes of the
# in-tree and round-start libraries, the default bench line, and the configs[4] trace.
# Stops at the first failing step.
# Usage (GPU box): bash tools/gpu_r04h.sh <tag>
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
  [ $rc -eq 0 ] || { tail -30 "$out/$name.log"; exit $rc; }
}
line() {  # line <label> <bench args...>
  local label=$1; shift
  printf "%s " "$label" >> $out/lines.log
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $out/tmp.json 2>> $out/bench_err.log || { echo "bench $label failed"; tail -5 $out/bench_err.log; exit 1; }
  tail -1 $out/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), json.dumps(d.get('kernel_ms')))" >> $out/lines.log
}
for r in 1 2; do
  ESLAM_GPU_LIB=$PWD/$L/lib_base.so line "maps_base" --local-maps --steps 20 --warmup 5
  line "maps_cur" --local-maps --steps 20 --warmup 5
  ESLAM_GPU_LIB=$PWD/$L/lib_nok1box.so line "maps_nok1box" --local-maps --steps 20 --warmup 5
  ESLAM_GPU_LIB=$PWD/$L/lib_nobox.so line "maps_nobox" --local-maps --steps 20 --warmup 5
done
cut -c1-300 $out/lines.log
step profile 600 bash tools/profile.sh $tag --steps 50 --warmup 10
step pmc 400 bash tools/pmc.sh $tag --steps 20 --warmup 5
step pmc_base 400 env ESLAM_GPU_LIB=$PWD/$L/lib_base.so bash tools/pmc.sh ${tag}_base --steps 20 --warmup 5
step bench 300 python bench.py
tail -1 $out/bench.log | cut -c1-400
step profile_maps 600 bash tools/profile.sh ${tag}_maps --local-maps --steps 10 --warmup 3
