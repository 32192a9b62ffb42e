#!/bin/bash
# Training-step probe through gpurun: each argument group (quoted) is one configuration of dnet's
# switches; per group a timing run and a rocprofv3 kernel trace (gpurun_out/tp_<i>_prof).
#   gpurun -- bash tools/gpu_runs/train_probe.sh "" "WGRAD_STREAM=0" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  timeout -k 10 200 python3 -u tools/train_probe.py $cfg --steps 30 >> gpurun_out/tp.log 2>&1 || exit $?
  tail -1 gpurun_out/tp.log
  rm -rf gpurun_out/tp_${i}_prof
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp_${i}_prof -o run -- \
      python3 tools/train_probe.py $cfg --steps 30 > gpurun_out/tp_${i}_prof.log 2>&1 || exit $?
  i=$((i + 1))
done
