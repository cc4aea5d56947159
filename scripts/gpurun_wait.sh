#!/bin/bash
# Submit one gpurun call, resubmitting ONLY while the pool answers "no slot / no box" (rc 3: nothing
# ran, nothing charged).  Any other outcome (success, failure, timeout, refusal) ends the loop.
#   scripts/gpurun_wait.sh <log> <timeout_s> <command>
log=$1; t=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1; rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo "rc=$rc" >> "$log"
exit $rc
