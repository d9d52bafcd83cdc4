#!/bin/bash
# Round-4: the full GPU suite after the merge fix, then the configs[4] per-particle-maps line
# (round-start library vs in-tree) and the sharded path on one rank vs the one-GPU path.
# Test failures do not stop the script; a timeout, abort or crash (rc >= 124) does.
# Usage (GPU box): bash tools/gpu_r04g.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/$1
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
step pytest_gpu 700 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests
tail -5 $out/pytest_gpu.log
line() {  # line <label> <bench args...>: one JSON summary line into lines.log
  local label=$1; shift
  printf "%s " "$label" >> $out/lines.log
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $out/tmp.json 2>> $out/bench_err.log || { echo "bench $label failed"; tail -5 $out/bench_err.log; exit 1; }
  tail -1 $out/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), json.dumps(d.get('kernel_ms')), json.dumps(d.get('map_update')))" >> $out/lines.log
}
for r in 1 2; do
  ESLAM_GPU_LIB=$PWD/$L/lib_base.so line "maps_base" --local-maps --steps 20 --warmup 5
  line "maps_cur" --local-maps --steps 20 --warmup 5
done
for r in 1 2; do
  line "single_4m" --steps 30 --warmup 5
  line "sharded_4m" --sharded --steps 30 --warmup 5
done
cat $out/lines.log | cut -c1-400
