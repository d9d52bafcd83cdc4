#!/bin/bash
# round-5 check: the match tests, then a kernel trace of --local-maps --match
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r05m2
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_particle_maps.py tests/test_gpu_facade.py -k "match or facade" -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash tools/trace_kernels.sh r05match2 --local-maps --match --steps 10 --warmup 20
