#!/bin/bash
# Session-3 A/B on one box: the GPU tests of the layers / DNET / golden fixtures / training graph
# (8-MFMA-tile weight gradient, fused down3 -> nconv4), then variants/base_pkg against the in-tree
# package: backward layer times, the graphed training step, the fused vs separate down3 + nconv4
# launches and the bench's config-2 forward line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) exit $1;; esac; }
sel="tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py tests/test_gpu_train_graph.py"
timeout -k 10 600 python -u -m pytest $sel -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -rf > gpurun_out/s3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/s3_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for rep in 1 2; do
  for L in nconv2 down1; do
    b=$(cd variants/base_pkg && timeout -k 10 100 python3 tools/bwd_layer_bench.py $L 30 2>/dev/null | tail -1); fatal $?
    c=$(timeout -k 10 100 python3 tools/bwd_layer_bench.py $L 30 2>/dev/null | tail -1); fatal $?
    echo "base $b | cur $c"
  done
  b=$(cd variants/base_pkg && timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); fatal $?
  c=$(timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); fatal $?
  echo "base $b | cur $c"
  b3=$(cd variants/base_pkg && timeout -k 10 60 python3 tools/fwd_layer_bench.py down3 50 2>/dev/null | tail -1); fatal $?
  b4=$(cd variants/base_pkg && timeout -k 10 60 python3 tools/fwd_layer_bench.py nconv4 50 2>/dev/null | tail -1); fatal $?
  c34=$(timeout -k 10 60 python3 tools/fwd_layer_bench.py down3_nconv4 50 2>/dev/null | tail -1); fatal $?
  echo "base $b3 + $b4 | cur $c34"
done
args="--alt-math= --no-config5 --no-train --no-guided --no-guided-train --no-cpu-baseline --steps 20"
for rep in 1 2; do
  for who in base cur; do
    dir=.; [ $who = base ] && dir=variants/base_pkg
    (cd $dir && timeout -k 10 300 python3 -u bench.py $args > $GRAFT_REPO_ROOT/gpurun_out/s3_bench_$who.log 2>&1); fatal $?
    tail -1 gpurun_out/s3_bench_$who.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$who fwd', d['value'], d['layer_us'])"
  done
done
exit $rc
