#!/bin/bash
# Weight-gradient stream priority (dnet.WGRAD_STREAM_PRIORITY 0 / -1) x library (in-tree / dp1),
# graphed and eager training steps, alternated; then the -1 timeline with dp1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prio
for rep in 1 2; do
  for V in base dp1; do
    lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
    for P in 0 -1; do
      echo -n "$V "; NCONV_LIB=$lib timeout -k 10 120 python3 tools/train_probe.py WGRAD_STREAM_PRIORITY=$P --steps 60 2>/dev/null || exit 1
      echo -n "$V "; NCONV_LIB=$lib timeout -k 10 120 python3 tools/train_probe.py --eager WGRAD_STREAM_PRIORITY=$P --steps 30 2>/dev/null || exit 1
    done
  done
done
rm -rf gpurun_out/prio/prof
NCONV_LIB=$PWD/variants/dp1/libnconv.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prio/prof -o run -- \
    python3 tools/train_probe.py WGRAD_STREAM_PRIORITY=-1 --steps 30 > gpurun_out/prio/prof.log 2>&1 || exit 1
