#!/bin/bash
# Dense weight-gradient A/B: tests, the wgrad microbench and the guided training leg with the
# in-tree library against variants/$1, alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
alt=${1:-prev}
mkdir -p gpurun_out/wab
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_gpu_dense_train.py tests/test_gpu_guided.py > gpurun_out/wab/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/wab/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for V in new $alt; do
    lib=""; [ $V != new ] && lib=$PWD/variants/$V/libnconv.so
    NCONV_LIB=$lib DENSE_OPS=wgrad timeout -k 10 120 python3 tools/dense_microbench.py "conv" 2>/dev/null | sed "s/^/$V /"
    NCONV_LIB=$lib timeout -k 10 300 python3 bench.py --no-train --no-config5 --no-guided --no-cpu-baseline \
        --alt-math "" --head-density 0 > gpurun_out/wab/bench_${V}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['guided_train_fwd_bwd_adamw']; print(sys.argv[2], 'guided train', d['ms_per_step'], d['fp32_mfma_frac'])" gpurun_out/wab/bench_${V}_$rep.json $V
  done
done
