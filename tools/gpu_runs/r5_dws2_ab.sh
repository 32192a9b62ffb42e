#!/bin/bash
# Guided training: the dense weight gradients' side stream joined per autograd node (1) or once at
# the end of the backward pass (2, NCONV_DENSE_WGRAD_STREAM): tests under 2, then the bench's guided
# training leg alternated (graphed + eager).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dws2
NCONV_DENSE_WGRAD_STREAM=2 timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_guided.py tests/test_gpu_dense_train.py > gpurun_out/dws2/pytest.log 2>&1
rc=$?; echo "tests (2): $(tail -1 gpurun_out/dws2/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for N in 2 1; do
    NCONV_DENSE_WGRAD_STREAM=$N timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided \
        --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/dws2/bench_${N}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); g=d['guided_train_fwd_bwd_adamw']
print('dense wgrad stream', sys.argv[2], g['frames_per_sec'], g['ms_per_step'], g['fp32_mfma_frac'], 'eager', g.get('eager'))" gpurun_out/dws2/bench_${N}_$rep.json $N
  done
done
