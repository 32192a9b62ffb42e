#!/bin/bash
# Kernel breakdown of the config-4 guided training step (eager, 3 timed steps after 2 warm-up).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof -o run -- \
    python3 tools/guided_train_driver.py 3 > gpurun_out/gprof.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/gprof.log; exit $rc
