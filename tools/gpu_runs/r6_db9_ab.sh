#!/bin/bash
# Round 6: the bench's guided legs (config 3 / 4, default dense math) per library arm, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/db9
tag=$1; shift
for rep in 1 2; do
  for arm in "$@"; do
    env $arm timeout -k 10 400 python3 bench.py --no-train --no-config5 --no-cpu-baseline --alt-math "" --head-density 0 \
        --guided-alt-math "" --steps 10 --warmup 3 > gpurun_out/db9/ab_${tag}.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); g=d['guided_fwd']; t=d['guided_train_fwd_bwd_adamw']
print(sys.argv[2], 'cfg3', g['ms_per_step'], 'cfg4', t['ms_per_step'], 'eager', t['eager']['ms_per_step'], 'dnet', d['value'])" gpurun_out/db9/ab_${tag}.json "$arm"
  done
done | tee gpurun_out/db9/ab_$tag.log
