#!/bin/bash
# Round 6: kernel-trace timeline of the config-4 guided training step (eager driver).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gtl
tag=$1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gtl/p_$tag -o run -- \
    python3 tools/guided_train_driver.py 4 > gpurun_out/gtl/log_$tag.txt 2>&1 || exit $?
f=$(find gpurun_out/gtl/p_$tag -name '*kernel_trace.csv' | head -1)
python3 tools/guided_timeline.py "$f" | tee gpurun_out/gtl/tl_$tag.txt
rm -rf gpurun_out/gtl/p_$tag
