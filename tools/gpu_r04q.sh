#!/bin/bash
# Round 4: configs[4] steady-state kernel trace + PMC passes (30 warm-up steps, 10 timed).
# Usage (GPU box): bash tools/gpu_r04q.sh <tag>
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out/$tag
timeout -k 10 900 bash tools/profile.sh ${tag}_maps --local-maps --steps 10 --warmup 30 > gpurun_out/$tag/profile_maps.log 2>&1
echo "== profile_maps rc=$?" | tee -a gpurun_out/$tag/session.log
