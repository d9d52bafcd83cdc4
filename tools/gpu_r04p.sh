#!/bin/bash
# Round 4: the full GPU suite and smoke at HEAD, the default bench line, and a kernel trace
# of the sharded path at 4M on one rank (RCCL).  Stops at a crash or timeout (rc >= 124).
# Usage (GPU box): bash tools/gpu_r04p.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
out=gpurun_out/$tag
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $out/session.log
  [ $rc -lt 124 ] || { tail -30 "$out/$name.log"; exit $rc; }
  return 0
}
step pytest_gpu 700 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests
tail -2 $out/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py
tail -1 $out/bench.log | cut -c1-300
step bench_sharded 300 python bench.py --sharded --no-cpu-baseline --steps 30 --warmup 5
step bench_single 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5
step trace_sharded 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_sharded -o run -- python3 bench.py --sharded --no-cpu-baseline --steps 30 --warmup 5
