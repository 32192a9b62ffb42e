#!/bin/bash
# The default bench line (all legs), then a rocprofv3 kernel trace of the same command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r4full_bench.log 2>&1 || { echo "bench rc=$?"; exit 1; }
tail -1 gpurun_out/r4full_bench.log > gpurun_out/r4full_bench.json
if [ "${PROF:-1}" = 1 ]; then
  rm -rf gpurun_out/r4full_prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4full_prof -o run -- python3 bench.py \
     > gpurun_out/r4full_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
  tail -1 gpurun_out/r4full_prof.log > gpurun_out/r4full_prof_line.json
fi
echo done
