#!/bin/bash
# DNET training backward: the layers' weight gradients round-robin over two side streams
# (NCONV_WGRAD_STREAMS 2) vs one (1): training tests under 2, the graphed / eager step alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wgs
NCONV_WGRAD_STREAMS=2 timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_train_launches.py tests/test_gpu_dnet.py tests/test_gpu_golden.py tests/test_gpu_train_graph.py \
    > gpurun_out/wgs/pytest.log 2>&1
rc=$?; echo "tests (2): $(tail -1 gpurun_out/wgs/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for N in 2 1; do
    timeout -k 10 120 python3 tools/train_probe.py WGRAD_STREAMS_N=$N --steps 60 2>/dev/null || exit 1
  done
done
for N in 2 1; do
  timeout -k 10 120 python3 tools/train_probe.py --eager WGRAD_STREAMS_N=$N --steps 30 2>/dev/null || exit 1
done
