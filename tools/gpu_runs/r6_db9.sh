#!/bin/bash
# Round 6: the 3x3 stride-1 dense convolutions with exact products on the bf16 matrix cores
# (NCONV_DENSE_MATH=bf16x9): dense / guided tests under it, per-shape microbench, then the bench's
# guided legs alternated against the fp32-MFMA default.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/db9
tag=$1; tests=${2:-tests/test_gpu_dense.py tests/test_gpu_dense_train.py tests/test_gpu_guided.py}
NCONV_DENSE_MATH=${TEST_MATH:-bf16x9} timeout -k 10 900 python -u -m pytest $tests -m gpu -q -x --timeout 400 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/db9/pytest_$tag.log 2>&1
rc=$?; tail -n 15 gpurun_out/db9/pytest_$tag.log
case $rc in 0|1) ;; *) exit $rc;; esac
for arm in ${ARMS:-fp32 bf16x9}; do
  NCONV_DENSE_MATH=$arm DENSE_OPS=fwd,dgrad timeout -k 10 120 python3 -u tools/dense_microbench.py "conv 64->32,conv 32->32,conv 128->64,conv 64->64" \
      2>&1 | sed "s|^|$arm |" || exit 1
done | tee gpurun_out/db9/micro_$tag.log
for rep in 1 2; do
  for arm in ${ARMS:-fp32 bf16x9}; do
    NCONV_DENSE_MATH=$arm timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-cpu-baseline \
        --alt-math "" --head-density 0 --steps 10 --warmup 3 > gpurun_out/db9/bench_${arm}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); g=d['guided_fwd']; t=d['guided_train_fwd_bwd_adamw']
print('math', sys.argv[2], 'cfg3', g['ms_per_step'], 'cfg4', t['ms_per_step'], 'eager', t['eager']['ms_per_step'], 'dnet', d['value'])" gpurun_out/db9/bench_${arm}_$rep.json $arm
  done
done | tee gpurun_out/db9/ab_$tag.log
