#!/bin/bash
# Round 6: dense_conv_bf9 variants, per-shape microbench (fwd + dgrad) per library arm.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/db9
tag=$1; shift
for arm in "$@"; do
  env $arm DENSE_OPS=fwd,dgrad timeout -k 10 120 python3 -u tools/dense_microbench.py "conv 64->32,conv 32->32,conv 128->64,conv 64->64" \
      2>&1 | grep -v amdgpu.ids | sed "s|^|$arm |" || exit 1
done | tee gpurun_out/db9/micro_$tag.log
