#!/bin/bash
# Round 6: forward A/B (fwd_probe.py, alternating arms) + kernel-trace timelines of the replayed
# forward for each arm.  gpurun --timeout 600 -- bash tools/gpu_runs/r6_fwd_tl.sh TAG "armA" "armB" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fwdtl
tag=$1; shift
for rep in 1 2 3; do
  for arm in "$@"; do
    timeout -k 10 120 python3 -u tools/fwd_probe.py $arm --steps 400 || exit $?
  done
done 2>&1 | tee gpurun_out/fwdtl/ab_$tag.log
i=0
for arm in "$@"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fwdtl/p_${tag}_$i -o run -- \
      python3 -u tools/fwd_probe.py $arm --steps 100 > /dev/null 2>&1 || exit $?
  f=$(find gpurun_out/fwdtl/p_${tag}_$i -name '*kernel_trace.csv' | head -1)
  echo "== arm $i: $arm" >> gpurun_out/fwdtl/tl_$tag.txt
  python3 tools/fwd_timeline.py "$f" >> gpurun_out/fwdtl/tl_$tag.txt || exit $?
  rm -rf gpurun_out/fwdtl/p_${tag}_$i
done
grep -E "span|==" gpurun_out/fwdtl/tl_$tag.txt
