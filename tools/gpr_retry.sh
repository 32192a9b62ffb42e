#!/bin/bash
# usage: gpr.sh OUTFILE TIMEOUT CMD   -- retries only on gpurun exit 3 (no box / infra transient)
out=$1; to=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1; rc=$?
  echo "exit $rc (attempt $i)" >> $out
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
