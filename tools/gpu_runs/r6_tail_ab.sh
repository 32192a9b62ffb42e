#!/bin/bash
# Round 6: the composed tail's tests, isolated tail vs composed-tail launches, and the forward A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tab
tag=${1:-t}
timeout -k 10 300 python -u -m pytest tests/test_gpu_tail_comp.py -m gpu -q -x --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/tab/pytest_$tag.log 2>&1 || { tail -20 gpurun_out/tab/pytest_$tag.log; exit 1; }
tail -1 gpurun_out/tab/pytest_$tag.log
for rep in 1 2 3; do
  for L in tail tailc; do timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 50 2>&1 | grep us || exit 1; done
done
for rep in 1 2 3; do
  for arm in compose_tail=1 compose_tail=0; do
    timeout -k 10 120 python3 -u tools/fwd_probe.py $arm --steps 400 2>&1 | grep forward || exit 1
  done
done
