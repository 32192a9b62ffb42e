#!/bin/bash
# Training forward in two batch slices on two streams (dnet.TRAIN_FWD_STREAMS 2 vs 1): the bitwise
# and parity tests, the graphed / eager step alternated, the two-stream step's timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tfs
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_train_launches.py tests/test_gpu_dnet.py tests/test_gpu_golden.py tests/test_gpu_train_graph.py \
    tests/test_gpu_dp.py > gpurun_out/tfs/pytest.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/tfs/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for N in 2 1; do
    timeout -k 10 120 python3 tools/train_probe.py TRAIN_FWD_STREAMS=$N --steps 60 2>/dev/null || exit 1
  done
done
for N in 2 1; do
  timeout -k 10 120 python3 tools/train_probe.py --eager TRAIN_FWD_STREAMS=$N --steps 30 2>/dev/null || exit 1
done
rm -rf gpurun_out/tfs/prof
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tfs/prof -o run -- \
    python3 tools/train_probe.py --steps 30 > gpurun_out/tfs/prof.log 2>&1 || exit 1
