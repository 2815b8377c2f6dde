#!/bin/bash
# Run gpurun, retrying only when the box could not be prepared (status=transient,
# nothing ran, nothing charged).  Usage: scripts/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  echo "$out" | tail -60
  if echo "$out" | grep -q "status=transient"; then sleep 45; continue; fi
  exit 0
done
