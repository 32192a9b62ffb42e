#!/bin/bash
# Round 6: per-shape microbench of given shapes (tools/dense_microbench.py name substrings) per arm.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/db9
tag=$1; shapes=$2; shift 2
for rep in 1 2; do
  for arm in "$@"; do
    env $arm DENSE_OPS=${OPS:-fwd} timeout -k 10 120 python3 -u tools/dense_microbench.py "$shapes" \
        2>&1 | grep -v amdgpu.ids | sed "s|^|$arm |" || exit 1
  done
done | tee gpurun_out/db9/micro2_$tag.log
