#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/fp32_rates > gpurun_out/fp32_rates.log 2>&1 || exit $?
cat gpurun_out/fp32_rates.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2a -o run -- python3 bench.py --no-cpu-baseline --no-guided-train > gpurun_out/prof_r2a.log 2>&1 || exit $?
echo prof ok
