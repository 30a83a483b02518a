#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool answers "no box / slot free" (exit 3:
# nothing ran, nothing charged); any other outcome (success, failure, refusal) ends the loop.
#   bash tools/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TMO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
