#!/bin/bash
# Backward check: layer / DNET / golden gradient tests, then the training-step bench leg + profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py -k backward -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_bwd.log 2>&1
rc=$?; echo "pytest layers rc=$rc"; grep -E "g_w \[|passed|failed" gpurun_out/pytest_bwd.log | tail -30
case $rc in 124|134|137|139) exit $rc;; esac
EXTRA_TESTS="tests/test_export.py" PROF=${PROF:-1} bash tools/_train.sh
