#!/bin/bash
# gpurun with retries while the pool has no free box (exit 3 / transient); any other outcome ends it.
# Usage: bash tools/gpurun_retry.sh <log> <timeout> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
  sleep 90
done
exit 3
