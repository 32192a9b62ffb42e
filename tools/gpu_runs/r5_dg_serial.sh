#!/bin/bash
# nconv2's input gradient alone (weight gradients on the main stream too): base vs variants/oa1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dgs
for rep in 1 2; do
  for V in base oa1; do
    lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
    echo -n "$V serial "; NCONV_LIB=$lib timeout -k 10 120 python3 tools/train_probe.py WGRAD_STREAM=0 --steps 60 2>/dev/null || exit 1
  done
done
for V in base oa1; do
  lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
  rm -rf gpurun_out/dgs/prof_$V
  NCONV_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dgs/prof_$V -o run -- \
      python3 tools/train_probe.py WGRAD_STREAM=0 --steps 20 > gpurun_out/dgs/prof_$V.log 2>&1 || exit 1
done
