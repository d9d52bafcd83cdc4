#!/bin/bash
# local-maps step: kernel trace + instruction counters of the merge
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/lmp3; mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t -o run -- python3 bench.py --local-maps --steps 6 --warmup 2 --no-cpu-baseline > $o/t.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $o/p -o run -- python3 bench.py --local-maps --steps 3 --warmup 1 --no-cpu-baseline > $o/p.log 2>&1
