#!/bin/bash
# Round 6: r6_iter.sh (tests + bench), then r6_fwd_tl.sh's forward A/B when the tests ran to the end
# (passed or failed, no fault).  gpurun -- bash tools/gpu_runs/r6_combo.sh TAG "tests" "armA" "armB"
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; tests=$2; shift 2
bash tools/gpu_runs/r6_iter.sh "$tag" "$tests"
rc=$?
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_runs/r6_fwd_tl.sh "$tag" "$@" || exit $?
exit $rc
