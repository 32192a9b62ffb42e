#!/bin/bash
# Development iteration through gpurun: selected GPU tests, then the short bench (config-2 forward +
# training step only), then a rocprofv3 kernel trace of that bench. Stops at the first failure.
#   gpurun -- bash tools/gpu_runs/iter.sh TAG "pytest selection" [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; sel=$2; shift 2
if [ -n "$sel" ]; then
  timeout -k 10 400 python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/it_${tag}_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/it_${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
args="--alt-math= --no-config5 --no-guided --no-guided-train --no-cpu-baseline $*"
timeout -k 10 300 python -u bench.py $args > gpurun_out/it_${tag}_bench.log 2>&1
rc=$?; tail -1 gpurun_out/it_${tag}_bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/it_${tag}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/it_${tag}_prof -o run -- \
    python3 bench.py $args --steps 20 > gpurun_out/it_${tag}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
