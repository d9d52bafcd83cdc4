#!/bin/bash
# Round-4 debugging + measurement on one GPU box.  Test steps may fail (assertions) without
# stopping the script; a timeout, abort or crash (rc >= 124) stops it.
# Usage (GPU box): bash tools/gpu_r04f.sh <tag>
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
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step maps_single 600 $PT tests/test_gpu_particle_maps.py
grep -E "PASSED|FAILED|Error" $out/maps_single.log | cut -c1-200 | tail -15
step maps_dist 400 $PT tests/test_gpu_dist.py -k maps
grep -E "PASSED|FAILED" $out/maps_dist.log | cut -c1-200 | tail -10
step maps_dist_nobox 400 env ESLAM_GPU_LIB=$PWD/$L/lib_nobox.so $PT tests/test_gpu_dist.py -k "maps and 3000"
grep -E "PASSED|FAILED" $out/maps_dist_nobox.log | cut -c1-200 | tail -5
for n in 4194304 262144; do
  for r in 1 2; do
    for lib in base cnt grp grp4; do
      printf "n=%s %s " $n $lib >> $out/ab.log
      ESLAM_GPU_LIB=$PWD/$L/lib_$lib.so timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --particles $n \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d['kernel_ms'])" >> $out/ab.log \
        || { echo "bench $lib failed"; exit 1; }
    done
  done
done
cut -c1-230 $out/ab.log
ESLAM_GPU_LIB=$PWD/$L/lib_stamps.so timeout -k 10 120 python tools/stamps.py 4194304 8 > $out/stamps_4m.log 2>&1 || { echo "stamps 4M failed"; tail -5 $out/stamps_4m.log; exit 1; }
cat $out/stamps_4m.log
ESLAM_GPU_LIB=$PWD/$L/lib_stamps.so timeout -k 10 120 python tools/stamps.py 262144 8 > $out/stamps_256k.log 2>&1 || { echo "stamps 256k failed"; exit 1; }
cat $out/stamps_256k.log
