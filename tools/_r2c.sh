#!/bin/bash
# Round-2 GPU check: whole GPU test suite (no -x, so every failure shows), smoke, bench line.
# Stops at the first fatal status (timeout / abort / segfault / kill).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_r2c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_r2c.log
fatal $rc && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2c.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_r2c.log
fatal $rc && exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r2c.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_r2c.log
exit $rc
