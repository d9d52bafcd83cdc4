#!/bin/bash
# per-particle maps: the new parity test and the configs[4] 1-GPU bench
cd "$(dirname "$0")/.."
o=gpurun_out/lm; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_particle_maps.py > $o/pytest.log 2>&1; rc=$?; tail -5 $o/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --local-maps --steps 20 --warmup 5 > $o/bench_lm.json 2> $o/bench_lm.err || { tail $o/bench_lm.err; exit 1; }
cat $o/bench_lm.json
timeout -k 10 300 python bench.py --rough --steps 50 --warmup 10 --no-cpu-baseline > $o/bench_rough.json 2> $o/bench_rough.err && cat $o/bench_rough.json
