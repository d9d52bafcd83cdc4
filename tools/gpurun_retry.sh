#!/bin/bash
# gpurun with a retry when no box was acquired (status=transient: pod busy or the box failed
# while being prepared; nothing ran and nothing was charged).  A run that started is never
# repeated.  Waits as long as gpurun's back-off asks ("retry in Ns").
# Usage: bash tools/gpurun_retry.sh <log> <timeout> '<command>' [attempts]
log=$1; t=$2; cmd=$3; attempts=${4:-14}
cd "$(dirname "$0")/.."
for attempt in $(seq 1 $attempts); do
  # every attempt snapshots the tree: the in-tree library must match the sources then (an
  # edit since the last build would fail the library's build-id check on the box)
  until timeout 900 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1; do sleep 60; done
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "run [1-9]" "$log"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
    wait_s=${wait_s:-120}
    [ "$wait_s" -lt 120 ] && wait_s=120
    echo "attempt $attempt: transient, retrying in $((wait_s + 15))s" >> "$log.retries"
    sleep $((wait_s + 15))
    continue
  fi
  exit $rc
done
exit 3
