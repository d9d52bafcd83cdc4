#!/bin/bash
# Round-4 K3 residency experiments: the full-size parity tests with each variant library, then
# interleaved bench lines at 4M, 1M and 256k.  Stops at the first failing step.
# Usage (GPU box): bash tools/gpu_r04i.sh <tag> <variant>...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
L=slam-eslam_amd/lib/ab
# the map merge's key signature (lib_msig): per-particle-map parity, then configs[4] lines
timeout -k 10 300 env ESLAM_GPU_LIB=$PWD/$L/lib_msig.so python -u -m pytest -q -x --timeout 240 --timeout-method thread \
  tests/test_gpu_particle_maps.py tests/test_gpu_dist.py -k "maps or particle" > $out/parity_msig.log 2>&1
rc=$?
echo "== parity msig rc=$rc" | tee -a $out/session.log
[ $rc -eq 0 ] || { tail -20 $out/parity_msig.log; exit $rc; }
for r in 1 2; do
  for v in main msig; do
    printf "maps %s " $v >> $out/ab.log
    timeout -k 10 200 env ESLAM_GPU_LIB=$PWD/$L/lib_$v.so python bench.py --local-maps --steps 20 --warmup 5 --no-cpu-baseline \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['kernel_ms']))" >> $out/ab.log \
      || { echo "maps bench $v failed"; exit 1; }
  done
done
for v in ${PARITY:-$@}; do
  timeout -k 10 400 env ESLAM_GPU_LIB=$PWD/$L/lib_$v.so python -u -m pytest -q -x --timeout 240 --timeout-method thread \
    tests/test_gpu_fullsize.py tests/test_gpu_dist.py > $out/parity_$v.log 2>&1
  rc=$?
  echo "== parity $v rc=$rc" | tee -a $out/session.log
  [ $rc -eq 0 ] || { tail -20 $out/parity_$v.log; exit $rc; }
done
for n in 4194304 1048576 262144; do
  for r in 1 2; do
    for v in "$@"; do
      printf "n=%s %s " $n $v >> $out/ab.log
      timeout -k 10 120 env ESLAM_GPU_LIB=$PWD/$L/lib_$v.so python bench.py --steps 30 --warmup 5 --no-cpu-baseline --particles $n \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['kernel_ms']))" >> $out/ab.log \
        || { echo "bench $v failed"; exit 1; }
    done
  done
done
for r in 1 2; do
  for v in "$@"; do
    printf "sharded n=4194304 %s " $v >> $out/ab.log
    timeout -k 10 120 env ESLAM_GPU_LIB=$PWD/$L/lib_$v.so python bench.py --sharded --steps 30 --warmup 5 --no-cpu-baseline --particles 4194304 \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d['kernel_ms']))" >> $out/ab.log \
      || { echo "sharded bench $v failed"; exit 1; }
  done
done
cut -c1-260 $out/ab.log
