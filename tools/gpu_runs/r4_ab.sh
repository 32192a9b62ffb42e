#!/bin/bash
# Same-box A/B of single-layer forward times: the baseline package copy in variants/base_pkg
# (an earlier commit's Python package + library) against the in-tree one, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
layers=${AB_LAYERS:-head down1 tail}
for rep in 1 2; do
  for L in $layers; do
    b=$(cd variants/base_pkg && timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 50 2>/dev/null | tail -1); r=$?
    case $r in 124|134|137|139) exit $r;; esac
    c=$(timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 50 2>/dev/null | tail -1); r=$?
    case $r in 124|134|137|139) exit $r;; esac
    echo "base $b | cur $c"
  done
done
