#!/bin/bash
# gpurun with a retry when no box was acquired (status=transient: pod busy or the box failed
# while being prepared; nothing ran and nothing was charged).  A run that started is never
# repeated.  Usage: bash tools/gpurun_retry.sh <log> <timeout> '<command>'
log=$1; t=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "run [1-9]" "$log"; then
    echo "attempt $attempt: transient, retrying" >> "$log.retries"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3
