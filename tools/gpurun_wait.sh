#!/bin/bash
# Run one gpurun call, retrying only while the pool has no free box (gpurun
# exit 3: nothing ran, nothing charged).  Any other outcome ends the loop.
# usage: tools/gpurun_wait.sh <log> <timeout_s> '<command>'
log=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && ! grep -q "no free box right now" "$log" && break
  sleep 90
done
echo "gpurun_wait rc=$rc tries=$i" >> "$log"
