#!/bin/bash
# Targeted GPU check: the given pytest selection, then the f9 gradient dump (tools/f9_dump.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf \
    > gpurun_out/pytest_check.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_check.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/f9_dump.py > gpurun_out/f9_dump.log 2>&1
src=$?; echo "f9_dump rc=$src"; tail -4 gpurun_out/f9_dump.log
exit $(( rc != 0 ? rc : src ))
