#!/bin/bash
# Kernel breakdown of the config-3 guided forward (tools/guided_driver.py under rocprofv3).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/gfwd
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gfwd -o run -- \
    python3 tools/guided_driver.py 5 > gpurun_out/gfwd.log 2>&1
rc=$?; echo "gfwd rc=$rc"; exit $rc
