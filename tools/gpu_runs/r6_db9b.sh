#!/bin/bash
# Round 6: dense maths through the ABI field (default bf16x9): dense / guided GPU tests, then the
# bench's guided legs with the other maths beside them (other_dense_math), twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/db9
tag=$1; tests=${2-tests/test_gpu_dense.py tests/test_gpu_dense_train.py tests/test_gpu_guided.py}
if [ -n "$tests" ]; then
  timeout -k 10 900 python -u -m pytest $tests -m gpu -q -x --timeout 400 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/db9/pytest_$tag.log 2>&1
  rc=$?; tail -n 5 gpurun_out/db9/pytest_$tag.log
  [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  timeout -k 10 400 python3 bench.py --no-train --no-config5 --no-cpu-baseline --alt-math "" --head-density 0 \
      --steps 10 --warmup 3 > gpurun_out/db9/benchb_${tag}_$rep.json 2>gpurun_out/db9/benchb_${tag}_$rep.err || exit 1
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); g=d['guided_fwd']; t=d['guided_train_fwd_bwd_adamw']
print('cfg3', g['dense_math'], g['ms_per_step'], {k: v['ms_per_step'] for k, v in g['other_dense_math'].items()})
print('cfg4', t['dense_math'], t['ms_per_step'], 'eager', t['eager']['ms_per_step'], {k: v['ms_per_step'] for k, v in t['other_dense_math'].items()})
print('dnet', d['value'])" gpurun_out/db9/benchb_${tag}_$rep.json
done | tee gpurun_out/db9/abb_$tag.log
