#!/bin/bash
# gpurun with waits while no box is free (exit 3: nothing ran, nothing charged).
# usage: tools/gpuq.sh LOG TIMEOUT CMD   (runs here, not on the box)
log=$1; to=$2; shift 2
for i in $(seq 1 ${GPUQ_TRIES:-60}); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
