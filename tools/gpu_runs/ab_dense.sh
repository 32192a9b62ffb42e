#!/bin/bash
# Dense-conv variants (libnconv builds under _exp/<name>/): forward time per shape
#   gpurun -- bash tools/gpu_runs/ab_dense.sh "v1 v2" "shape-substring,..."
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in $1; do
  NCONV_LIB=_exp/$v/libnconv.so DENSE_FWD_ONLY=${FWD_ONLY:-1} timeout -k 10 300 python3 tools/dense_microbench.py "$2" 2>/dev/null | sed "s/^/$v /" || exit $?
done
