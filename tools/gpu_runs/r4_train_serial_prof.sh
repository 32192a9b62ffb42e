#!/bin/bash
# Kernel trace of the graphed config-2 training step with every weight gradient on the main stream
# (WGRAD_STREAM=0: kernels run one at a time, so the trace gives each kernel's standalone time),
# then of the default two-stream step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/tser_prof gpurun_out/tdef_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tser_prof -o run -- \
    python3 tools/train_probe.py WGRAD_STREAM=0 --steps 20 > gpurun_out/tser_prof.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tdef_prof -o run -- \
    python3 tools/train_probe.py --steps 20 > gpurun_out/tdef_prof.log 2>&1 || exit $?
tail -1 gpurun_out/tser_prof.log; tail -1 gpurun_out/tdef_prof.log
