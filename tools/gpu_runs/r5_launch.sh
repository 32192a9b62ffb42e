#!/bin/bash
# Training-step launch trimming: the new and affected GPU tests, the A/B of the graphed step
# (merged prologue + cropped tail on / off), and the default step's kernel timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    ${R5_TESTS:-tests/test_gpu_train_launches.py tests/test_gpu_dnet.py tests/test_gpu_golden.py tests/test_gpu_fused_bwd.py} \
    ${R5_TESTS2-tests/test_gpu_dp.py tests/test_gpu_train_graph.py} > gpurun_out/r5_launch_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5_launch_pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "" "DNET.merged_prologue=0 DNET.crop_in_tail=0" "" "DNET.merged_prologue=0 DNET.crop_in_tail=0"; do
    timeout -k 10 120 python3 tools/train_probe.py $a --steps 50 || exit $?
done > gpurun_out/r5_launch_ab.log 2>&1
cat gpurun_out/r5_launch_ab.log
rm -rf gpurun_out/tl_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tl_prof -o run -- \
    python3 tools/train_probe.py --steps 20 > gpurun_out/tl_prof.log 2>&1 || exit $?
python3 tools/step_timeline.py gpurun_out/tl_prof/run_kernel_trace.csv > gpurun_out/r5_train_step_timeline.txt
tail -3 gpurun_out/r5_train_step_timeline.txt
