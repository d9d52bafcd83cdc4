#!/bin/bash
# Round 4, for the next round's plan: configs[4] SQ instruction mix (map merge, K1 DELTA) and
# the K1 / K3 phase stamps at 4M and 256k with this round's kernels.
# Usage (GPU box): bash tools/gpu_r04u.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 120 env ESLAM_GPU_LIB=$PWD/slam-eslam_amd/lib/ab/lib_stamps.so python tools/stamps.py 4194304 8 > $out/stamps_4m.log 2>&1
echo "== stamps_4m rc=$?" | tee -a $out/session.log
timeout -k 10 120 env ESLAM_GPU_LIB=$PWD/slam-eslam_amd/lib/ab/lib_stamps.so python tools/stamps.py 262144 8 > $out/stamps_256k.log 2>&1
echo "== stamps_256k rc=$?" | tee -a $out/session.log
timeout -k 10 600 bash tools/pmc.sh ${tag}_maps --local-maps --steps 10 --warmup 30 > $out/pmc_maps.log 2>&1
echo "== pmc_maps rc=$?" | tee -a $out/session.log
