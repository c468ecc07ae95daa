#!/bin/bash
# Re-submit a gpurun call only when the infrastructure did not run it at all
# (status=transient: no box / box lost while preparing / backoff); a command
# that ran (any rc) is never re-submitted.  A backoff notice's "retry in Ns"
# is honoured.  Usage: gpurun_retry.sh OUT TIMEOUT CMD
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 25); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  if grep -q "status=transient rc=None" "$OUT" || grep -q "backing off" "$OUT"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$OUT" | tail -1 | grep -o "[0-9]*")
    sleep $(( ${wait_s:-80} + 10 ))
    continue
  fi
  break
done
