#!/bin/bash
# Dense forward-kernel iteration: dense / guided GPU tests, the dense microbenchmark (forward and
# input gradient) and the guided bench legs (config 3 / 4), for variants/base_pkg and in-tree.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${DENSE_TESTS:-tests/test_gpu_dense.py tests/test_gpu_dense_train.py tests/test_gpu_guided.py} \
    -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/dfwd_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/dfwd_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
args="--alt-math= --no-config5 --no-train --no-cpu-baseline --steps 10"
for who in base cur; do
  dir=.; [ $who = base ] && dir=variants/base_pkg
  (cd $dir && DENSE_OPS=fwd,dgrad timeout -k 10 300 python3 -u tools/dense_microbench.py > $GRAFT_REPO_ROOT/gpurun_out/dfwd_mb_$who.log 2>&1) || exit $?
  (cd $dir && timeout -k 10 400 python3 -u bench.py $args > $GRAFT_REPO_ROOT/gpurun_out/dfwd_bench_$who.log 2>&1) || exit $?
  echo "== $who"; grep -E "^fwd|^dgrad" gpurun_out/dfwd_mb_$who.log
  tail -1 gpurun_out/dfwd_bench_$who.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('guided', d['guided_fwd'], d['guided_train_fwd_bwd_adamw'])"
done
exit $rc
