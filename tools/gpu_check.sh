#!/bin/bash
# One GPU call: the -m gpu suite, then an interleaved A/B of library builds with BENCH_ARGS
# (bash tools/gpu_check.sh <tag> "<sizes>" lib...; PYTEST=0 skips the suite, TESTS="<paths>" and
# K="<-k expression>" narrow it)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; sizes=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
if [ "${PYTEST:-1}" = 1 ]; then
  timeout -k 10 ${PYTEST_LIMIT:-600} python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 \
    || { tail -40 $out/pytest_gpu.log; exit 1; }
  tail -2 $out/pytest_gpu.log
fi
[ $# -gt 0 ] || exit 0
timeout -k 10 600 bash tools/ab_libs.sh $tag/ab ${REPS:-3} "$sizes" "$@" > $out/ab.out 2>&1 || { tail -20 $out/ab.out; exit 1; }
grep "^n=" $out/ab/ab.log | cut -c1-200
