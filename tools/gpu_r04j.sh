#!/bin/bash
# Round 4: the full GPU suite and smoke at HEAD, interleaved lines (4M one-GPU and sharded,
# configs[4]) against the libraries before this round's last changes, K1 phase stamps, the
# default bench line, and the kernel trace + PMC passes at 4M and 256k.
# Stops at a crash or timeout (rc >= 124); test failures are reported and the script goes on.
# Usage (GPU box): bash tools/gpu_r04j.sh <tag>
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
  tail -1 $out/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), json.dumps(d.get('kernel_ms')))" >> $out/lines.log
}
step pytest_gpu 700 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests
tail -3 $out/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -1 $out/smoke.log
for r in 1 2; do
  line "4m_cur" "" --steps 30 --warmup 5
  line "4m_r04i" main --steps 30 --warmup 5
  line "4m_k1w6" k1w6 --steps 30 --warmup 5
  line "sharded4m_cur" "" --sharded --steps 30 --warmup 5
  line "maps_cur" "" --local-maps --steps 20 --warmup 5
  line "maps_dreg" dreg --local-maps --steps 20 --warmup 5
  line "maps_base" base --local-maps --steps 20 --warmup 5
done
cut -c1-300 $out/lines.log
step stamps_4m 120 env ESLAM_GPU_LIB=$PWD/$L/lib_stamps.so python tools/stamps.py 4194304 8
head -6 $out/stamps_4m.log
step bench 300 python bench.py
tail -1 $out/bench.log | cut -c1-300
step profile 600 bash tools/profile.sh $tag --steps 50 --warmup 10
step profile_256k 400 bash tools/profile.sh ${tag}_256k --particles 262144 --steps 50 --warmup 10
