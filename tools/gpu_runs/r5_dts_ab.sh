#!/bin/bash
# Guided training convolutions' forward in two batch slices on two streams (NCONV_DENSE_TRAIN_SLICES
# 2 vs 1): the bitwise test, then the bench's guided training leg alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dts
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_guided.py -k "sliced or graphed or f9" > gpurun_out/dts/pytest.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/dts/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for N in 2 1; do
    NCONV_DENSE_TRAIN_SLICES=$N timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided \
        --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/dts/bench_${N}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); g=d['guided_train_fwd_bwd_adamw']
print('train slices', sys.argv[2], g['frames_per_sec'], g['ms_per_step'], g['fp32_mfma_frac'], 'eager', g.get('eager'))" gpurun_out/dts/bench_${N}_$rep.json $N
  done
done
