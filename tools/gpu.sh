#!/bin/bash
# gpurun wrapper for development: re-submits only when the harness reports a transient box
# failure before the command ran (status "transient", nothing charged); any result of the
# command itself is returned as is.
for attempt in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[gpu.sh] transient/no box (attempt $attempt), waiting 60 s"
  sleep 60
done
exit $rc
