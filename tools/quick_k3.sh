#!/bin/bash
# Quick GPU check of a scan/segments change: parity subset, bench at 4M and 256k, region clocks.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/q
mkdir -p $o
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py > $o/pytest.log 2>&1; rc=$?; tail -3 $o/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for n in 4194304 262144; do
  timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --particles $n > $o/bench_$n.json 2>$o/bench_$n.err || exit $?
  python3 -c "import json; d=json.load(open('$o/bench_$n.json')); print($n, d['value'], d['ms_per_step'], d['kernel_ms'])"
done
L=$PWD/slam-eslam_amd/lib/libeslam_gpu_eslam_k1_prof.so
if [ -f $L ]; then
  for n in 4194304 262144; do
    N=$n ESLAM_GPU_LIB=$L timeout -k 10 120 python tools/k1_prof.py > $o/regions_$n.log 2>&1 || exit $?
    grep "^K3" $o/regions_$n.log
  done
fi
