#!/bin/bash
# Dense (guided) kernel iteration: guided / dense GPU tests, the dense microbenchmark and the
# config-4 guided training step, each for variants/base_pkg and the in-tree package.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${DENSE_TESTS:-tests/test_gpu_dense.py tests/test_gpu_dense_train.py tests/test_gpu_guided.py} \
    -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/dense_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/dense_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for who in base cur; do
  dir=.; [ $who = base ] && dir=variants/base_pkg
  (cd $dir && timeout -k 10 300 python3 -u tools/dense_microbench.py ${MB_SHAPES:-} > $GRAFT_REPO_ROOT/gpurun_out/dense_mb_$who.log 2>&1) || exit $?
  (cd $dir && timeout -k 10 300 python3 -u tools/guided_train_driver.py 5 > $GRAFT_REPO_ROOT/gpurun_out/dense_gt_$who.log 2>&1) || exit $?
  echo "== $who: $(tail -1 gpurun_out/dense_gt_$who.log)"; grep wgrad gpurun_out/dense_mb_$who.log
done
exit $rc
