#!/bin/bash
# Transposed weight-gradient row split: dense-training + guided tests, guided training A/B
# (NCONV_WGD_TR_ROWS=1 / 0 alternated), a kernel trace of the eager guided step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/trr
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_dense_train.py tests/test_gpu_guided.py > gpurun_out/trr/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/trr/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 1 0; do
    NCONV_WGD_TR_ROWS=$v timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided --no-cpu-baseline \
        --alt-math "" --head-density 0 > gpurun_out/trr/bench_${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['guided_train_fwd_bwd_adamw']; print('NCONV_WGD_TR_ROWS=' + sys.argv[2], d['ms_per_step'], d['fp32_mfma_frac'])" gpurun_out/trr/bench_${v}_$rep.json $v
  done
done
rm -rf gpurun_out/trr/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trr/prof -o run -- \
    python3 tools/guided_train_driver.py 3 > gpurun_out/trr/prof.log 2>&1
