#!/bin/bash
# Guided eval forward (config 3) in two batch slices on two streams (NCONV_GUIDED_STREAMS 2 vs 1):
# the bitwise / oracle tests, then the bench's guided forward leg alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gs
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_guided.py > gpurun_out/gs/pytest.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/gs/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for N in 2 1; do
    NCONV_GUIDED_STREAMS=$N timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided-train \
        --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/gs/bench_${N}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); g=d['guided_fwd']
print('guided streams', sys.argv[2], g['frames_per_sec'], g['ms_per_step'], g['fp32_mfma_frac'], 'dnet', d['value'])" gpurun_out/gs/bench_${N}_$rep.json $N
  done
done
