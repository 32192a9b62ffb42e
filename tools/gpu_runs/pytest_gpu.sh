#!/bin/bash
# Whole GPU test suite (no -x: every failure is listed), then smoke(). Usage via gpurun:
#   gpurun --timeout 1100 -- bash tools/gpu_runs/pytest_gpu.sh [TAG] [pytest args...]
# Log: gpurun_out/pytest_<TAG>.log, gpurun_out/smoke_<TAG>.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-all}; shift
args=${*:-tests}
git_rev=$(cat REVISION 2>/dev/null || echo unknown)
echo "revision $git_rev" > gpurun_out/pytest_$tag.log
timeout -k 10 900 python -u -m pytest $args -m gpu -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider -rf >> gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$tag.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1
src=$?; echo "smoke rc=$src"; tail -3 gpurun_out/smoke_$tag.log
exit $(( rc != 0 ? rc : src ))
