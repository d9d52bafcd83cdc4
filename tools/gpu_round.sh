#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first GPU fault/timeout.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>; exit codes 0/1 (test failures) continue, others stop
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > gpurun_out/gpu.txt 2>&1; nproc >> gpurun_out/gpu.txt; lscpu | grep "Model name" >> gpurun_out/gpu.txt
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testsall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchsharded) run bench_sharded 600 python bench.py --sharded --steps 20 --warmup 5 --no-cpu-baseline ;;
    benchfast) run bench 600 python bench.py --steps 50 --warmup 10 --no-cpu-baseline ;;
    benchshort) run bench 600 python bench.py --steps 20 --warmup 5 --cpu-steps 2 ;;
  esac
done
