#!/bin/bash
# Training-step probe: in-tree library and variants/wm2 (wgrad_mfma2 built in), each with the
# weight gradients on the side stream (default) and on the main stream (WGRAD_STREAM=0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for dir in . variants/wm2; do
    for sw in "" "WGRAD_STREAM=0"; do
      o=$(cd $dir && timeout -k 10 200 python3 -u tools/train_probe.py $sw --steps 40 2>/dev/null | tail -1); r=$?
      case $r in 124|134|137|139) exit $r;; esac
      echo "$dir: $o"
    done
  done
done
