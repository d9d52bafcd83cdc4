#!/bin/bash
# Round-end measurements on one GPU box: kernel-trace + PMC profile of the bench line, the
# instruction-mix passes, the bench line itself (with both CPU baselines), the other
# workloads, smoke and the GPU test suite.  Usage (GPU box): bash tools/round_measure.sh <tag> [a|b]
# (a: the profiles and the configs[1..3] bench lines; b: the other workloads, smoke and the
# tests; default both -- about 20 minutes, more than one gpurun call allows)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
part=${2:-ab}
out=gpurun_out/round_$tag
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>: stop at the first failure
  local name=$1 t=$2; shift 2
  echo "== $name" >> $out/session.log
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> $out/session.log
  [ $rc -eq 0 ] || { tail -20 "$out/$name.log"; exit $rc; }
}
rocm-smi --showproductname > $out/gpu_box.txt 2>&1; nproc >> $out/gpu_box.txt; lscpu | grep "Model name" >> $out/gpu_box.txt
if [[ $part == *a* ]]; then
step profile 900 bash tools/profile.sh $tag --steps 50 --warmup 10
step pmc 900 bash tools/pmc.sh $tag --steps 20 --warmup 5
step bench 600 python bench.py
step bench_256k 300 python bench.py --particles 262144 --steps 50 --warmup 10 --no-cpu-baseline
step bench_sharded 300 python bench.py --sharded --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline
step bench_2m 300 python bench.py --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline
step bench_sharded_b 300 python bench.py --sharded --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline
step bench_2m_b 300 python bench.py --particles 2097152 --steps 50 --warmup 10 --no-cpu-baseline
fi
if [[ $part == *b* ]]; then
step bench_16m 300 python bench.py --particles 16777216 --steps 20 --warmup 5 --no-cpu-baseline
step bench_rough 300 python bench.py --rough --steps 50 --warmup 10 --no-cpu-baseline
step bench_local_maps 600 python bench.py --local-maps --steps 20 --warmup 5
step bench_local_maps_steady 600 python bench.py --local-maps --steps 20 --warmup 30 --no-cpu-baseline
step prof_lm 900 bash tools/profile.sh ${tag}_lm --local-maps --steps 20 --warmup 30
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
fi
