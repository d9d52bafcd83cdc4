#!/bin/bash
# 256k latency diagnosis: K1 per-wave timeline and a kernel trace of the bench
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/d256; mkdir -p $o
[ -n "$TL" ] && N=262144 ESLAM_GPU_LIB=$PWD/slam-eslam_amd/lib/libeslam_gpu_eslam_k1_tl.so timeout -k 10 120 python tools/k1_timeline.py > $o/tl.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t -o run -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 --particles 262144 > $o/trace.log 2>&1
