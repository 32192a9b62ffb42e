#!/bin/bash
# Weight-prologue latency: tests, the prologue kernels' durations (rocprof) and forward bench lines,
# in-tree library against variants/prev (the previous revision), alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/proab
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_train_launches.py tests/test_gpu_dnet.py -k "prologue or launches or stream" \
    > gpurun_out/proab/pytest.log 2>&1
rc=$?; tail -1 gpurun_out/proab/pytest.log; [ $rc -eq 0 ] || exit $rc
for V in new prev; do
  lib=""; [ $V = prev ] && lib=$PWD/variants/prev/libnconv.so
  rm -rf gpurun_out/proab/pb_$V
  NCONV_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/proab/pb_$V -o run -- \
      python3 tools/prologue_bench.py 50 > gpurun_out/proab/pb_$V.log 2>&1 || exit $?
done
for rep in 1 2 3; do
  for V in on off; do
    sp=1; [ $V = off ] && sp=0
    NCONV_STREAM_PROLOGUE=$sp timeout -k 10 200 python3 bench.py --no-train --no-config5 --no-guided --no-guided-train \
        --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/proab/bench_${V}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/proab/bench_${V}_$rep.json "stream_prologue=$V"
  done
done
