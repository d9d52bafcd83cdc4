#!/bin/bash
# Round-4 check on one GPU box: the -m gpu suite at HEAD, the VALU issue-cost microbenchmark,
# then interleaved A/B of K1 variants (4M, 256k) and of configs[4] (base vs current).
# Usage (GPU box): bash tools/gpu_r04d.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
step() {  # step <name> <timeout> <cmd...>: stop at the first failure
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $out/session.log
  [ $rc -eq 0 ] || { tail -30 "$out/$name.log"; exit $rc; }
}
step ubench 60 tools/_build/ubench_valu
cat $out/ubench.log
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 $out/pytest_gpu.log
L=slam-eslam_amd/lib/ab
for n in 4194304 262144; do
  for r in 1 2; do
    for lib in base cnt grp grp4; do
      printf "n=%s %s " $n $lib >> $out/ab.log
      ESLAM_GPU_LIB=$PWD/$L/lib_$lib.so timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --particles $n \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d['kernel_ms'])" >> $out/ab.log \
        || { echo "bench $lib failed"; exit 1; }
    done
  done
done
cat $out/ab.log | cut -c1-160
for r in 1 2; do
  for lib in base grp; do
    printf "lm %s " $lib >> $out/ab_lm.log
    ESLAM_GPU_LIB=$PWD/$L/lib_$lib.so timeout -k 10 200 python bench.py --local-maps --steps 20 --warmup 5 --no-cpu-baseline \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d.get('map_update'))" >> $out/ab_lm.log \
      || { echo "bench lm $lib failed"; exit 1; }
  done
done
cat $out/ab_lm.log | cut -c1-400
ESLAM_GPU_LIB=$PWD/$L/lib_stamps.so timeout -k 10 120 python tools/stamps.py 4194304 8 > $out/stamps_4m.log 2>&1 || { echo "stamps 4M failed"; tail -5 $out/stamps_4m.log; exit 1; }
cat $out/stamps_4m.log
ESLAM_GPU_LIB=$PWD/$L/lib_stamps.so timeout -k 10 120 python tools/stamps.py 262144 8 > $out/stamps_256k.log 2>&1 || { echo "stamps 256k failed"; exit 1; }
cat $out/stamps_256k.log
