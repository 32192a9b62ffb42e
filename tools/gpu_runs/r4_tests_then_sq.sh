#!/bin/bash
# Full GPU suite + smoke (pytest_gpu.sh), then the counter probe (r4_sq.sh) unless a step faulted,
# aborted or timed out (test failures alone do not stop the probe).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_runs/pytest_gpu.sh "${1:-r4}"
rc=$?
case $rc in 0|1) ;; *) echo "stopping: rc=$rc"; exit $rc;; esac
bash tools/gpu_runs/r4_sq.sh
src=$?
exit $(( rc != 0 ? rc : src ))
