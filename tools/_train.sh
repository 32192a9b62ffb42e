#!/bin/bash
# Loss / training check: loss + golden + training GPU tests, then the training-step bench leg.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_golden.py tests/test_gpu_train_graph.py tests/test_gpu_dnet.py ${EXTRA_TESTS} -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_train.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --math fp32 --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline --steps 20 > gpurun_out/bench_train.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_train.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], json.dumps(d['train_fwd_bwd_adamw']))"
if [ "${PROF:-0}" = 1 ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- python3 bench.py --math fp32 --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline --steps 10 > gpurun_out/prof_train.log 2>&1 || exit $?
echo prof ok
fi
