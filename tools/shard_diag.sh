#!/bin/bash
# sharded-path overhead at configs[3]'s 2M per GPU on one rank: bench lines and a kernel trace
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/sd; mkdir -p $o
timeout -k 10 200 python bench.py --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline > $o/single.json 2>$o/single.err || exit 1
timeout -k 10 200 python bench.py --sharded --particles 2097152 --steps 50 --warmup 10 > $o/sharded.json 2>$o/sharded.err || exit 1
for f in single sharded; do python3 -c "import json; d=json.load(open('$o/$f.json')); print('$f', d['value'], d['ms_per_step'], d['kernel_ms'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t -o run -- python3 bench.py --sharded --particles 2097152 --steps 20 --warmup 5 > $o/t.log 2>&1
