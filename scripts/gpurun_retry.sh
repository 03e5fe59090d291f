#!/bin/bash
# Run one gpurun call, retrying only while gpurun reports that no box or slot
# was free (exit 3: nothing ran, nothing charged). Any other outcome -- the
# command ran, failed or timed out -- is returned as it is.
#   scripts/gpurun_retry.sh <timeout s> <log> '<command>'
T=$1; LOG=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box right now\|GPU slot(s) on this pod are busy" "$LOG"; then exit $rc; fi
  echo "gpurun_retry: no box (attempt $i), waiting" >&2
  sleep 120
done
exit 3
