#!/bin/bash
# Guided eval forward: step 1 (the DNET depth network) on its own stream beside the RGB encoders
# (NCONV_GUIDED_STEP1_STREAM 1 vs 0): the bitwise / oracle tests, then the bench's guided forward leg.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s1s
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_guided.py -k "streams or config3 or f5 or generalized" > gpurun_out/s1s/pytest.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/s1s/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for N in 1 0; do
    NCONV_GUIDED_STEP1_STREAM=$N timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided-train \
        --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/s1s/bench_${N}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); g=d['guided_fwd']
print('step1 stream', sys.argv[2], g['frames_per_sec'], g['ms_per_step'], g['fp32_mfma_frac'])" gpurun_out/s1s/bench_${N}_$rep.json $N
  done
done
