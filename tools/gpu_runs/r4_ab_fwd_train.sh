#!/bin/bash
# Same-box A/B of variants/base_pkg against the in-tree library: forward layers (AB_LAYERS) and the
# graphed training step, alternating; then the forward-only bench line of each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_LAYERS="${AB_LAYERS:-tail nconv5 head}" bash tools/gpu_runs/r4_ab.sh || exit $?
for rep in 1 2; do
  b=$(cd variants/base_pkg && timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); r=$?
  case $r in 124|134|137|139) exit $r;; esac
  c=$(timeout -k 10 200 python3 -u tools/train_probe.py --steps 40 2>/dev/null | tail -1); r=$?
  case $r in 124|134|137|139) exit $r;; esac
  echo "train base $b | cur $c"
done
args="--alt-math= --no-config5 --no-train --no-guided --no-guided-train --no-cpu-baseline"
for who in base cur; do
  dir=.; [ $who = base ] && dir=variants/base_pkg
  (cd $dir && timeout -k 10 300 python3 -u bench.py $args > $GRAFT_REPO_ROOT/gpurun_out/abf_bench_$who.log 2>&1) || exit $?
  tail -1 gpurun_out/abf_bench_$who.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$who fwd', d['value'], d['layer_us'])"
done
