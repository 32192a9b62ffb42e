#!/bin/bash
# Inference split probe: the config-2 forward line for several stream shares / stream counts.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
args="--alt-math= --no-config5 --no-train --no-guided --no-guided-train --no-cpu-baseline"
for rep in 1 2; do
  for v in "" "--inference-shares 5,3" "--inference-shares 3,5" "--inference-shares 6,2" "--inference-streams 3 --inference-shares 4,2,2" "--inference-streams 1"; do
    r=$(timeout -k 10 200 python3 -u bench.py $args $v 2>/dev/null | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit $?
    echo "[$v] $r"
  done
done
