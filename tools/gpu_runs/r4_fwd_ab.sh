#!/bin/bash
# Forward A/B on one box: forward GPU tests of the in-tree library, then single-layer forward
# times (tools/fwd_layer_bench.py) and the bench's config-2 forward line of variants/base_pkg and
# the in-tree package, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
sel=${FWD_TESTS:-tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py}
timeout -k 10 600 python -u -m pytest $sel -m gpu -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -rf > gpurun_out/fab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/fab_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
AB_LAYERS="${AB_LAYERS:-tail nconv5 down1 head}" bash tools/gpu_runs/r4_ab.sh || exit $?
args="--alt-math= --no-config5 --no-train --no-guided --no-guided-train --no-cpu-baseline --steps 20"
for rep in 1 2; do
  for who in base cur; do
    dir=.; [ $who = base ] && dir=variants/base_pkg
    (cd $dir && timeout -k 10 300 python3 -u bench.py $args > $GRAFT_REPO_ROOT/gpurun_out/fab_bench_$who.log 2>&1) || exit $?
    tail -1 gpurun_out/fab_bench_$who.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$who fwd', d['value'], d['layer_us'])"
  done
done
exit $rc
