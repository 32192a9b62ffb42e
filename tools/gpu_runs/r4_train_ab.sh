#!/bin/bash
# Training-step A/B: GPU tests of the training graph, then the graphed config-2 training step
# (tools/train_probe.py) of variants/base_pkg and of the in-tree package, alternating; then a
# kernel trace of the in-tree step (gpurun_out/tab_prof).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
sel=${TRAIN_TESTS:-tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py tests/test_gpu_train_graph.py}
timeout -k 10 600 python -u -m pytest $sel -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -rf > gpurun_out/tab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/tab_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for rep in 1 2; do
  b=$(cd variants/base_pkg && timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); r=$?
  case $r in 124|134|137|139) exit $r;; esac
  c=$(timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); r=$?
  case $r in 124|134|137|139) exit $r;; esac
  echo "base $b | cur $c"
done
rm -rf gpurun_out/tab_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tab_prof -o run -- \
    python3 tools/train_probe.py --steps 20 > gpurun_out/tab_prof.log 2>&1
prc=$?; echo "prof rc=$prc"
exit $rc
