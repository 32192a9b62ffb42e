#!/bin/bash
# Guided-model iteration through gpurun: guided GPU tests, the config-3/4 bench legs, a rocprofv3
# kernel trace of the config-4 leg.   gpurun -- bash tools/gpu_runs/iter_guided.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_guided.py tests/test_gpu_dense_train.py tests/test_gpu_dense.py \
    -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/itg_${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/itg_${tag}_pytest.log; [ $rc -eq 0 ] || exit $rc
args="--alt-math= --no-config5 --no-train --no-cpu-baseline"
timeout -k 10 400 python -u bench.py $args > gpurun_out/itg_${tag}_bench.log 2>&1
rc=$?; tail -1 gpurun_out/itg_${tag}_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/itg_${tag}_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/itg_${tag}_prof -o run -- \
    python3 bench.py $args --no-guided --steps 30 > gpurun_out/itg_${tag}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
