#!/bin/bash
# Full GPU suite + smoke, then the same-box layer A/B against variants/base_pkg.
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_runs/pytest_gpu.sh "${1:-r4}"
rc=$?
case $rc in 0|1) ;; *) echo "stopping: rc=$rc"; exit $rc;; esac
AB_LAYERS="head down1 down2 tail" bash tools/gpu_runs/r4_ab.sh
exit $rc
