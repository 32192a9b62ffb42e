#!/bin/bash
# Same-box A/B of single-layer forward times: tools/ab_layers.sh "layers" variantdir... (developer tool)
# Each variant dir holds a libnconv.so (tools/build_variant.sh); "cur" = the in-tree library.
cd "$GRAFT_REPO_ROOT" || exit 1
layers=$1; shift
for rep in 1 2; do
  for v in cur "$@"; do
    for L in $layers; do
      if [ "$v" = cur ]; then lib=""; else lib="$v/libnconv.so"; fi
      out=$(NCONV_LIB=$lib timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 50 2>/dev/null | tail -1)
      rc=$?
      echo "$v $L $out"
      case $rc in 124|134|137|139) exit $rc;; esac
    done
  done
done
