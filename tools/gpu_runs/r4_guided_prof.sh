#!/bin/bash
# Config-4 guided training step: wall time per step, then a rocprofv3 kernel trace of the same driver.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/guided_train_driver.py 6 > gpurun_out/gtrain_wall.log 2>&1 || exit $?
tail -1 gpurun_out/gtrain_wall.log
rm -rf gpurun_out/gtrain_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gtrain_prof -o run -- \
    python3 tools/guided_train_driver.py 4 > gpurun_out/gtrain_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
