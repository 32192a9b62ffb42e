#!/bin/bash
# Round 6: the headline forward (bench.py, forward legs only) per environment arm, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fab
tag=$1; shift
for rep in 1 2 3; do
  for arm in "$@"; do
    env $arm timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided --no-guided-train --no-cpu-baseline \
        --alt-math "" --head-density 0 > gpurun_out/fab/b_$tag.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], 'fps', d['value'], 'ms', d['ms_per_step'], 'down1', d['layer_us']['nconv_down1'], 'down2', d['layer_us']['nconv_down2'])" gpurun_out/fab/b_$tag.json "$arm"
  done
done | tee gpurun_out/fab/ab_$tag.log
