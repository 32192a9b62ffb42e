#!/bin/bash
# Double-buffered dense weight gradient: dense-training and guided GPU tests, then the guided
# training leg with NCONV_WGD_DB=1 / 0 alternated, then a kernel trace of the eager guided step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wgd
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_dense_train.py tests/test_gpu_guided.py > gpurun_out/wgd/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/wgd/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for db in 1 0; do
    NCONV_WGD_DB=$db timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided --no-cpu-baseline \
        --alt-math "" --head-density 0 > gpurun_out/wgd/bench_${db}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['guided_train_fwd_bwd_adamw']; print('NCONV_WGD_DB=' + sys.argv[2], d['ms_per_step'], d['fp32_mfma_frac'])" gpurun_out/wgd/bench_${db}_$rep.json $db
  done
done
for db in 1 0; do
  rm -rf gpurun_out/wgd/prof_$db
  NCONV_WGD_DB=$db timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wgd/prof_$db -o run -- \
      python3 tools/guided_train_driver.py 3 > gpurun_out/wgd/prof_$db.log 2>&1 || exit $?
done
