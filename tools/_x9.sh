#!/bin/bash
# bf16x9 check: targeted GPU tests, then a forward-only bench over the three arithmetics.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_products.py tests/test_gpu_layers.py tests/test_gpu_golden.py tests/test_gpu_dnet.py -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_x9.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "signed|positive|passed|failed|Error|error" gpurun_out/pytest_x9.log | tail -40
fatal $rc && exit $rc
timeout -k 10 300 python -u bench.py --no-train --no-guided --no-guided-train --no-cpu-baseline --steps 30 > gpurun_out/bench_x9.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/bench_x9.log
exit $rc
