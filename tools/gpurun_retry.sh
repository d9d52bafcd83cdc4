#!/bin/bash
# gpurun with a retry when no box was acquired (status=transient: pod busy or the box failed
# while being prepared; nothing ran and nothing was charged).  A run that started is never
# repeated.  Waits as long as gpurun's back-off asks ("retry in Ns").
# Usage: bash tools/gpurun_retry.sh <log> <timeout> '<command>' [attempts]
log=$1; t=$2; cmd=$3; attempts=${4:-14}
for attempt in $(seq 1 $attempts); do
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
