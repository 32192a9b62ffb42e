#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_guided.py tests/test_gpu_dense_train.py -m gpu -v -s --timeout 400 \
   --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_guided.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_guided.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_runs/r4_ab.sh
