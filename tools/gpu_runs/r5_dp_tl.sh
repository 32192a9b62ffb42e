#!/bin/bash
# Two-stream (default) training-step timelines, in-tree library vs variants/dp1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dptl
for V in base dp1; do
  lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
  rm -rf gpurun_out/dptl/prof_$V
  NCONV_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dptl/prof_$V -o run -- \
      python3 tools/train_probe.py --steps 30 > gpurun_out/dptl/prof_$V.log 2>&1 || exit 1
  tail -1 gpurun_out/dptl/prof_$V.log
done
