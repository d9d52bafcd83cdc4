#!/bin/bash
# One GPU session on the box: bash tools/gpu_session.sh <tag> <step>...
#   tests       every -m gpu test (one pytest process)
#   tests:<f>   the -m gpu tests of tests/<f>
#   smoke       __graft_entry__.smoke()
#   bench       bench.py defaults (configs[2], 4M)
#   bench256k   configs[1]
#   benchlm     --local-maps (configs[4]'s 8M per GPU)
#   benchsh     --sharded at configs[3]'s 2M per rank
#   proflm      rocprofv3 kernel trace + FETCH/WRITE/VALUBusy passes of --local-maps
#   prof        the same for the default bench
# Logs go to gpurun_out/<tag>/.  A step that times out, aborts or faults ends the session.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
run() {  # run <name> <timeout> <cmd...>; 0/1 (test failures) continue, anything else stops
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $out/session.log
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $out/session.log
  tail -4 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
prof() {  # prof <name> <bench args...>
  local name=$1; shift
  run ${name}_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$name/trace -o run -- python3 bench.py --no-cpu-baseline "$@"
  for c in FETCH_SIZE WRITE_SIZE VALUBusy; do
    run ${name}_$c 300 rocprofv3 --pmc $c --output-format csv -d $out/$name/$c -o run -- python3 bench.py --no-cpu-baseline "$@"
  done
}
rocm-smi --showproductname > $out/gpu.txt 2>&1; nproc >> $out/gpu.txt; lscpu | grep "Model name" >> $out/gpu.txt
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 1150 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    tests:*) f=${step#tests:}; run pytest_${f%.py} 900 python -u -m pytest tests/$f -m gpu -v --timeout 900 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 300 python bench.py --steps 50 --warmup 10 --cpu-steps 8 ;;
    bench256k) run bench256k 300 python bench.py --particles 262144 --steps 50 --warmup 10 --no-cpu-baseline ;;
    benchlm) run benchlm 300 python bench.py --local-maps --steps 20 --warmup 5 --no-cpu-baseline ;;
    benchsh) run benchsh 300 python bench.py --sharded --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline ;;
    proflm) prof proflm --local-maps --steps 20 --warmup 5 ;;
    prof) prof prof --steps 50 --warmup 10 ;;
  esac
done
