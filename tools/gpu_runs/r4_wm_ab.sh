#!/bin/bash
# Weight-gradient A/B: GPU tests of the backward, then per-layer backward times
# (tools/bwd_layer_bench.py) and the graphed training step (tools/train_probe.py) of
# variants/base_pkg and of the in-tree package, alternating on one box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
sel=${TRAIN_TESTS:-tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py tests/test_gpu_train_graph.py}
timeout -k 10 600 python -u -m pytest $sel -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -rf > gpurun_out/wm_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/wm_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for rep in 1 2; do
  for L in ${AB_LAYERS:-nconv2 down1 nconv6 nconv5}; do
    b=$(cd variants/base_pkg && timeout -k 10 100 python3 tools/bwd_layer_bench.py $L 30 2>/dev/null | tail -1); r=$?
    case $r in 124|134|137|139) exit $r;; esac
    c=$(timeout -k 10 100 python3 tools/bwd_layer_bench.py $L 30 2>/dev/null | tail -1); r=$?
    case $r in 124|134|137|139) exit $r;; esac
    echo "base $b | cur $c"
  done
  b=$(cd variants/base_pkg && timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); r=$?
  case $r in 124|134|137|139) exit $r;; esac
  c=$(timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); r=$?
  case $r in 124|134|137|139) exit $r;; esac
  echo "base $b | cur $c"
done
exit $rc
