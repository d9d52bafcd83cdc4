#!/bin/bash
# The round's bench lines on one GPU box (each step under its own time limit, stop at the first
# failure): bash tools/round_lines.sh <tag>   -> gpurun_out/lines_<tag>/*.log
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/lines_$1
mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1 || { echo "$name rc=$?"; tail -5 "$out/$name.log"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
}
step bench 400 python bench.py
step bench_256k 200 python bench.py --particles 262144 --steps 50 --warmup 10 --no-cpu-baseline
step bench_2m 200 python bench.py --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline
step bench_sharded_2m 200 python bench.py --sharded --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline
step bench_sharded_4m 200 python bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline
step bench_4m_b 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline
step bench_16m 300 python bench.py --particles 16777216 --steps 20 --warmup 5 --no-cpu-baseline
step bench_rough 200 python bench.py --rough --steps 50 --warmup 10 --no-cpu-baseline
step bench_local_maps 400 python bench.py --local-maps --steps 20 --warmup 5
step bench_local_maps_steady 300 python bench.py --local-maps --steps 20 --warmup 30 --no-cpu-baseline
step bench_local_maps_match 300 python bench.py --local-maps --match --steps 20 --warmup 10 --no-cpu-baseline
step bench_local_maps_600 400 python bench.py --local-maps --scan-patches 600 --map-pages 40 --steps 5 --warmup 3
step_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo smoke ok || { echo "smoke rc=$?"; tail -5 $out/smoke.log; exit 1; }; }
step_smoke
