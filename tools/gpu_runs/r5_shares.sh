#!/bin/bash
# Inference split shares / streams sweep on one box (forward-only bench lines, alternated).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/shares
for rep in 1 2; do
  for cfg in "2 1,1" "2 5,3" "2 3,5" "3 3,3,2" "3 2,3,3"; do
    set -- $cfg
    timeout -k 10 200 python3 bench.py --no-train --no-config5 --no-guided --no-guided-train --no-cpu-baseline \
        --alt-math "" --head-density 0 --inference-streams $1 --inference-shares $2 \
        > gpurun_out/shares/b_$1_$2_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
        gpurun_out/shares/b_$1_$2_$rep.json "streams=$1 shares=$2"
  done
done
