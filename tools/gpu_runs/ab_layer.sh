#!/bin/bash
# Per-layer timing of library variants: gpurun -- bash tools/gpu_runs/ab_layer.sh "v1 v2 ..." "layer1 layer2"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in $1; do
  for l in $2; do
    NCONV_LIB=_exp/$v/libnconv.so timeout -k 10 120 python -u tools/fwd_layer_bench.py $l 30 2>/dev/null | sed "s/^/$v /" || exit $?
  done
done
