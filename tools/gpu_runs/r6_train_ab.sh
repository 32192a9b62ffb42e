#!/bin/bash
# Round 6: graphed config-2 training step A/B (tools/train_probe.py arms, alternating, 3 rounds),
# then kernel-trace timelines of each arm's replayed step (tools/step_timeline.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/trab
tag=$1; shift
for rep in 1 2 3; do
  for arm in "$@"; do
    timeout -k 10 120 python3 -u tools/train_probe.py $arm --steps 30 2>&1 | grep "train step" || exit 1
  done
done | tee gpurun_out/trab/ab_$tag.log
i=0
for arm in "$@"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trab/p_${tag}_$i -o run -- \
      python3 -u tools/train_probe.py $arm --steps 10 > /dev/null 2>&1 || exit $?
  f=$(find gpurun_out/trab/p_${tag}_$i -name '*kernel_trace.csv' | head -1)
  echo "== arm $i: $arm" >> gpurun_out/trab/tl_$tag.txt
  python3 tools/step_timeline.py "$f" >> gpurun_out/trab/tl_$tag.txt || exit $?
  rm -rf gpurun_out/trab/p_${tag}_$i
done
grep -E "span|==" gpurun_out/trab/tl_$tag.txt
