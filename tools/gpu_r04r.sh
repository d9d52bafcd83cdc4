#!/bin/bash
# Round 4: interleaved lines at 256k and 1M (in-tree library vs no LDS window below 512k vs
# two-item K3 tiles at 256k), then the configs[4] steady-state kernel trace and byte counters.
# Usage (GPU box): bash tools/gpu_r04r.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
out=gpurun_out/$tag
mkdir -p $out
L=slam-eslam_amd/lib/ab
line() {  # line <label> <lib or ""> <bench args...>
  local label=$1 lib=$2; shift 2
  printf "%s " "$label" >> $out/ab.log
  if [ -n "$lib" ]; then export ESLAM_GPU_LIB=$PWD/$L/lib_$lib.so; else unset ESLAM_GPU_LIB; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $out/tmp.json 2>> $out/bench_err.log || { echo "bench $label failed"; tail -5 $out/bench_err.log; exit 1; }
  unset ESLAM_GPU_LIB
  tail -1 $out/tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], json.dumps(d.get('kernel_ms')))" >> $out/ab.log
}
for r in 1 2 3; do
  for n in 262144 1048576; do
    line "n=$n head" "" --particles $n --steps 30 --warmup 5
    line "n=$n nowin" nowin --particles $n --steps 30 --warmup 5
    line "n=$n k3i2" k3i2 --particles $n --steps 30 --warmup 5
  done
done
cut -c1-200 $out/ab.log
p=gpurun_out/prof_${tag}_maps
mkdir -p $p
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p/trace -o run -- python3 bench.py --no-cpu-baseline --local-maps --steps 10 --warmup 30 > $p/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $p/fetch -o run -- python3 bench.py --no-cpu-baseline --local-maps --steps 10 --warmup 30 > $p/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $p/write -o run -- python3 bench.py --no-cpu-baseline --local-maps --steps 10 --warmup 30 > $p/write.log 2>&1 && \
python3 tools/prof_summary.py $p > $p/summary.json
echo "== maps profile rc=$?" | tee -a $out/session.log
