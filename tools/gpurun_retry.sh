#!/bin/bash
# Submit a gpurun call, resubmitting ONLY while the pool reports no free box / slot (status
# "transient", nothing ran, nothing charged).  Any call that ran -- pass or fail -- is final.
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient rc=None" "$LOG"; then sleep 200; continue; fi
  exit $rc
done
