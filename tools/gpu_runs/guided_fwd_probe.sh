#!/bin/bash
# Guided forward probe through gpurun: dense-kernel microbench per shape, then a rocprofv3 kernel
# trace of the config-3 leg alone (gpurun_out/gfp_prof).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/dense_microbench.py > gpurun_out/gfp_micro.log 2>&1 || exit $?
cat gpurun_out/gfp_micro.log
rm -rf gpurun_out/gfp_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gfp_prof -o run -- \
    python3 bench.py --alt-math= --no-config5 --no-train --no-guided-train --no-cpu-baseline --steps 10 \
    > gpurun_out/gfp_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
