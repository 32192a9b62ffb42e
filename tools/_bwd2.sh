#!/bin/bash
# Backward check: layer backward tests (every bwd_math), per-layer backward timing fp32 vs bf16x3,
# kernel trace of the bf16 backward kernels, then the training tests and the training-step bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { case $1 in 124|134|137|139) echo "fatal rc=$1"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py -k backward -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_bwd.log 2>&1
rc=$?; echo "pytest layers rc=$rc"; grep -E "passed|failed|Error" gpurun_out/pytest_bwd.log | tail -12
stop $rc
[ $rc = 0 ] || exit $rc
for L in nconv2 down1 nconv6 nconv5; do for M in fp32 bf16x3; do
  NCONV_BWD_MATH=$M timeout -k 10 60 python3 tools/bwd_layer_bench.py $L 10 || exit $?
done; done
for L in nconv2 nconv6; do
  NCONV_BWD_MATH=bf16x3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ktbw_$L -o run -- python3 tools/bwd_layer_bench.py $L 5 > gpurun_out/ktbw_$L.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_golden.py tests/test_gpu_train_graph.py tests/test_gpu_dnet.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_train.log 2>&1
rc=$?; echo "pytest train rc=$rc"; tail -4 gpurun_out/pytest_train.log
stop $rc
timeout -k 10 300 python -u bench.py --math fp32 --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline --steps 20 > gpurun_out/bench_train.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_train.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], json.dumps(d['train_fwd_bwd_adamw']))"
