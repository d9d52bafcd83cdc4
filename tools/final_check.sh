#!/bin/bash
# One GPU call at the end of a work session: the -m gpu suite as the driver runs it, smoke,
# the default bench line, and interleaved single / sharded-path runs at 4M per rank.
# Usage (GPU box): bash tools/final_check.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>: stop at the first failure
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> $out/session.log
  [ $rc -eq 0 ] || { tail -20 "$out/$name.log"; exit $rc; }
}
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step bench_sharded_4m 200 python bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline
step bench_4m_b 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline
step bench_sharded_4m_b 200 python bench.py --sharded --steps 50 --warmup 10 --no-cpu-baseline
