#!/bin/bash
# Re-submit a gpurun call only when the infrastructure did not run it at all
# (status=transient: no box / box lost while preparing / backoff); a command
# that ran (any rc) is never re-submitted.  Usage: gpurun_retry.sh OUT TIMEOUT CMD
OUT=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  if grep -q "status=transient rc=None" "$OUT" || grep -q "backing off" "$OUT"; then
    sleep 90
    continue
  fi
  break
done
