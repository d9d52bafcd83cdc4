#!/bin/bash
# Region clocks (ESLAM_K1_PROF build) + a rocprofv3 kernel trace of a short bench run.
# Usage (GPU box): bash tools/quick_prof.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/$tag
if [ -f slam-eslam_amd/lib/libeslam_gpu_eslam_k1_prof.so ]; then
  ESLAM_GPU_LIB=$PWD/slam-eslam_amd/lib/libeslam_gpu_eslam_k1_prof.so timeout -k 10 120 python tools/k1_prof.py > gpurun_out/$tag/regions.log 2>&1 || exit 1
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/trace -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/$tag/trace.log 2>&1 || exit 1
python3 - "$tag" <<'PY'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/{tag}/trace/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:48]:48s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.2f} us")
PY
