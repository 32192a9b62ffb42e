#!/bin/bash
# Round 6: the row-pair weight gradient (wgrad_mfma2): its tests, then graphed training-step A/B
# over environment arms (alternating, 3 rounds), then a kernel-trace timeline of the first arm.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wm2
tag=$1; tests=$2; shift 2
if [ -n "$tests" ]; then
  timeout -k 10 600 python -u -m pytest $tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/wm2/pytest_$tag.log 2>&1
  rc=$?; tail -n 3 gpurun_out/wm2/pytest_$tag.log
  [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2 3; do
  for arm in "$@"; do
    env $arm timeout -k 10 120 python3 -u tools/train_probe.py --steps 30 2>&1 | grep "train step" | sed "s|^|$arm |" || exit 1
  done
done | tee gpurun_out/wm2/ab_$tag.log
arm=$1
env $arm timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wm2/p_$tag -o run -- \
    python3 -u tools/train_probe.py --steps 10 > /dev/null 2>&1 || exit $?
f=$(find gpurun_out/wm2/p_$tag -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/wm2/tl_$tag.txt || exit $?
rm -rf gpurun_out/wm2/p_$tag
grep -E "span|wgrad_mfma" gpurun_out/wm2/tl_$tag.txt | cut -c1-120
