#!/bin/bash
# Round 6: forward tests, then the graphed config-2 forward A/B over environment arms (alternating, 3
# rounds) and isolated head launches.  gpurun -- bash tools/gpu_runs/r6_fwd_ab.sh TAG "tests" armA armB
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fab
tag=$1; tests=$2; shift 2
if [ -n "$tests" ]; then
  timeout -k 10 600 python -u -m pytest $tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/fab/pytest_$tag.log 2>&1
  rc=$?; tail -n 2 gpurun_out/fab/pytest_$tag.log
  [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2 3; do
  for arm in "$@"; do
    env $arm timeout -k 10 120 python3 -u tools/fwd_probe.py --steps 400 2>&1 | grep forward | sed "s|^|$arm |" || exit 1
    env $arm timeout -k 10 60 python3 -u tools/fwd_layer_bench.py head 30 2>&1 | grep us | sed "s|^|$arm |" || exit 1
  done
done | tee gpurun_out/fab/ab_$tag.log
