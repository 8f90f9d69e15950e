#!/bin/bash
# Run one gpurun call, retrying only while the pool has no box or slot free
# (a transient status: nothing ran, nothing was charged).  Any run that
# reached the GPU -- passed or failed -- ends the loop.
#   bash tools/gpurun_retry.sh LOG TIMEOUT_S 'COMMAND'
LOG=$1; T=$2; CMD=$3
for attempt in $(seq 1 40); do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$LOG" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${wait_s:-150} + 10 ))
    continue
  fi
  echo "attempt $attempt rc=$rc" >> "$LOG"
  exit $rc
done
exit 3
