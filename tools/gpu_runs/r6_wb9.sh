#!/bin/bash
# Round 6: the split-bf16 dense weight gradient: its training tests, the wgrad microbench (fp32 vs
# bf16x9), then the bench's guided legs against a build without it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wb9
tag=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense_train.py -m gpu -q -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/wb9/pytest_$tag.log 2>&1
rc=$?; tail -n 4 gpurun_out/wb9/pytest_$tag.log; [ $rc -eq 0 ] || exit $rc
for arm in fp32 bf16x9; do
  NCONV_DENSE_MATH=$arm DENSE_OPS=wgrad timeout -k 10 120 python3 -u tools/dense_microbench.py "${WSHAPES:-conv 64->32,conv 32->32,conv 128->64,conv 64->64}" \
      2>&1 | grep -v amdgpu.ids | sed "s|^|$arm |" || exit 1
done | tee gpurun_out/wb9/micro_$tag.log
bash tools/gpu_runs/r6_db9_ab.sh wb9_$tag "NCONV_X=1" "NCONV_LIB=_exp/nowb9/libnconv.so"
