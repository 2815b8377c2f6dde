#!/bin/bash
# Run gpurun, retrying only when the box could not be prepared or the pool is
# backing off (status=transient / exit 3: nothing ran, nothing charged); waits
# the back-off gpurun names.  Usage: scripts/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 ${TRIES:-12}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out" | tail -60
  if [ $rc -eq 3 ] || echo "$out" | grep -q "status=transient"; then
    w=$(echo "$out" | grep -o "retry in [0-9]*s" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-90} + 15 ))
    continue
  fi
  exit $rc
done
exit 3
