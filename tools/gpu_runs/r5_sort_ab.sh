#!/bin/bash
# Head: nconv1's halo pixels sorted by tap count. Head / layer / training parity tests, then the
# forward (both densities) and the training step alternated: in-tree library vs variants/base.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sort
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_golden.py tests/test_gpu_dnet.py tests/test_gpu_train_launches.py tests/test_gpu_layers.py \
    > gpurun_out/sort/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/sort/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for V in new base; do
    lib=""; [ $V = base ] && lib=$PWD/variants/base/libnconv.so
    NCONV_LIB=$lib timeout -k 10 200 python3 bench.py --no-config5 --no-guided --no-guided-train \
        --no-cpu-baseline --alt-math "" > gpurun_out/sort/bench_${V}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); h=d['head_density']
print(sys.argv[2], d['value'], 'head5', h['0.05']['kernel_us'], 'head40', h['0.40']['kernel_us'], 'train_ms', d['train_fwd_bwd_adamw']['ms_per_step'])" gpurun_out/sort/bench_${V}_$rep.json $V
  done
done
