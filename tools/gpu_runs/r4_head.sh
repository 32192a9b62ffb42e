#!/bin/bash
# Head iteration: the head / golden / DNET GPU tests, same-box A/B of the head against
# variants/base_pkg, then a forward-only bench line (base, then current).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${HEAD_TESTS:-tests} -m gpu -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/head_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/head_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
AB_LAYERS="${AB_LAYERS:-head down1 down2}" bash tools/gpu_runs/r4_ab.sh || exit $?
args="--alt-math= --no-config5 --no-train --no-guided --no-guided-train --no-cpu-baseline"
(cd variants/base_pkg && cp ../../bench.py . && timeout -k 10 300 python -u bench.py $args > ../../gpurun_out/head_bench_base.log 2>&1) || exit $?
timeout -k 10 300 python -u bench.py $args > gpurun_out/head_bench_cur.log 2>&1 || exit $?
for f in base cur; do echo "$f: $(tail -1 gpurun_out/head_bench_$f.log | cut -c1-200)"; done
exit $rc
