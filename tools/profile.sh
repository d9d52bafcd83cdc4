#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.
# Usage (on the GPU box): bash tools/profile.sh <tag> [bench args...]
cd "$(dirname "$0")/.."
tag=$1; shift
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p $out
args="$@"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu-baseline $args > $out/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $out/trace.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 bench.py --no-cpu-baseline $args > $out/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -20 $out/fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- python3 bench.py --no-cpu-baseline $args > $out/write.log 2>&1 || { echo "write rc=$?"; tail -20 $out/write.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc VALUBusy --output-format csv -d $out/valu -o run -- python3 bench.py --no-cpu-baseline $args > $out/valu.log 2>&1 || { echo "valu rc=$?"; tail -20 $out/valu.log; }
timeout -k 10 600 rocprofv3 --pmc VALUUtilization --output-format csv -d $out/valuutil -o run -- python3 bench.py --no-cpu-baseline $args > $out/valuutil.log 2>&1 || { echo "valuutil rc=$?"; tail -20 $out/valuutil.log; }
find $out -name "*.csv" | head -20
python3 tools/prof_summary.py $out > $out/summary.json && cat $out/summary.json
