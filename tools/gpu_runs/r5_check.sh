#!/bin/bash
# Round-5 check: the whole GPU suite + smoke (pytest_gpu.sh), then one bench line.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_runs/r5_check.sh TAG [pytest args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-r5}; shift
bash tools/gpu_runs/pytest_gpu.sh "$tag" "$@"
rc=$?
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
brc=$?; echo "bench rc=$brc"; tail -3 gpurun_out/bench_$tag.err
exit $(( rc != 0 ? rc : brc ))
