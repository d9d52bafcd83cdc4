#!/bin/bash
# The full GPU suite at HEAD, then interleaved bench lines of the in-tree library ("cur")
# against variant libraries (slam-eslam_amd/lib/ab/lib_<v>.so) at 4M, 1M and 256k, and the
# sharded path at 4M.  Stops at a crash or timeout (rc >= 124) or a failing bench.
# Usage (GPU box): SIZES="4194304 262144" bash tools/gpu_ab.sh <tag> <variant>...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
L=slam-eslam_amd/lib/ab
timeout -k 10 700 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $out/pytest_gpu.log 2>&1
rc=$?
echo "== pytest_gpu rc=$rc" | tee -a $out/session.log
tail -2 $out/pytest_gpu.log
[ $rc -lt 124 ] || exit $rc
line() {  # line <label> <lib or ""> <bench args...>
  local label=$1 lib=$2; shift 2
  printf "%s " "$label" >> $out/ab.log
  if [ -n "$lib" ]; then export ESLAM_GPU_LIB=$PWD/$L/lib_$lib.so; else unset ESLAM_GPU_LIB; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $out/tmp.json 2>> $out/bench_err.log || { echo "bench $label failed"; tail -5 $out/bench_err.log; exit 1; }
  unset ESLAM_GPU_LIB
  tail -1 $out/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d.get('kernel_ms')))" >> $out/ab.log
}
for n in ${SIZES:-4194304 1048576 262144}; do
  for r in 1 2; do
    line "n=$n cur" "" --particles $n --steps 30 --warmup 5
    for v in "$@"; do line "n=$n $v" $v --particles $n --steps 30 --warmup 5; done
  done
done
if [ -z "$NO_SHARDED" ]; then
  for r in 1 2; do
    line "sharded cur" "" --sharded --steps 30 --warmup 5
    for v in "$@"; do line "sharded $v" $v --sharded --steps 30 --warmup 5; done
  done
fi
cut -c1-260 $out/ab.log
