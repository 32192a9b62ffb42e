#!/bin/bash
# The tail's input gradient (dgrad_phase) with its stager one plane ahead (variants/dp1: 79 instead
# of 109 VGPRs) against the in-tree library: parity tests on dp1, the graphed and the serial
# training step alternated, the kernel alone under rocprof (serial step).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dp
NCONV_LIB=$PWD/variants/dp1/libnconv.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 \
    --timeout-method thread -m gpu tests/test_gpu_dnet.py -k "train or tail" tests/test_gpu_golden.py \
    tests/test_gpu_train_launches.py tests/test_gpu_layers.py > gpurun_out/dp/pytest.log 2>&1
rc=$?; echo "dp1: $(tail -1 gpurun_out/dp/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for V in base dp1; do
    lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
    echo -n "$V "; NCONV_LIB=$lib timeout -k 10 120 python3 tools/train_probe.py --steps 60 2>/dev/null || exit 1
    echo -n "$V serial "; NCONV_LIB=$lib timeout -k 10 120 python3 tools/train_probe.py WGRAD_STREAM=0 --steps 60 2>/dev/null || exit 1
  done
done
for V in base dp1; do
  lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
  rm -rf gpurun_out/dp/prof_$V
  NCONV_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dp/prof_$V -o run -- \
      python3 tools/train_probe.py WGRAD_STREAM=0 --steps 20 > gpurun_out/dp/prof_$V.log 2>&1 || exit 1
done
