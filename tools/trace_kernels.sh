cd /root/repo
export TMPDIR=/tmp
out=gpurun_out/tr_$1
mkdir -p $out
shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu-baseline "$@" > $out/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $out/trace.log; exit 1; }
python3 tools/prof_summary.py $out > $out/summary.json && python3 -c "
import json,sys; d=json.load(open('$out/summary.json'))['kernels']
for k,v in sorted(d.items(), key=lambda kv:-kv[1].get('pct',0))[:25]: print(f\"{k:40s} calls {v.get('calls')} avg_us {v.get('avg_us',0):10.1f} pct {v.get('pct',0):5.1f}\")"
