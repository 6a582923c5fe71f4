#!/bin/bash
# gpurun, retried only while the pool has no free box (status=transient: nothing ran, nothing
# was charged).  Usage: bash tools/gpurun_wait.sh <log> <timeout-seconds> '<command>'
LOG=$1; T=$2; shift 2
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  grep -q "status=transient" "$LOG" || exit 0
  sleep 150
done
