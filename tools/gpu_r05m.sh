#!/bin/bash
# round-5 check: the match tests, the sharded maps scenario, the no-window A/B and the
# --local-maps --match line (each step under its own limit, stop at the first failure)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/r05m
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_particle_maps.py tests/test_gpu_dist.py -k "match or maps" -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 200 python bench.py --local-maps --match --steps 10 --warmup 10 --no-cpu-baseline > $out/lm_match.log 2>&1 || { tail -10 $out/lm_match.log; exit 1; }
tail -c 600 $out/lm_match.log
PYTEST=0 REPS=2 bash tools/gpu_check.sh r05m/nowin "262144 1048576 4194304" slam-eslam_amd/lib/libeslam_gpu.so slam-eslam_amd/lib/ab/lib_nowin.so
