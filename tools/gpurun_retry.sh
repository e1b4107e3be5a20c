#!/bin/bash
# Local helper (this container, not the GPU box): run one gpurun call, retrying only when gpurun
# reports that no box was obtained (exit 3: nothing ran, nothing charged).  Usage:
#   bash tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $out 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "attempt $i: no box (rc 3), waiting" >> $out.retries
  sleep 90
done
exit 3
