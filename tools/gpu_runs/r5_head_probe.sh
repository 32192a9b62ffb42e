#!/bin/bash
# Head kernel phase probes (timing only, wrong results): B=8 352x1216 head launch time with the
# in-tree library and with nconv2's data sums / nconv1's taps / the pooled copies compiled out.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for V in base non2 non1 nopool; do
    lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
    r=$(NCONV_LIB=$lib timeout -k 10 60 python3 tools/fwd_layer_bench.py head 50 2>/dev/null | tail -1) || exit 1
    echo "$V $r"
  done
done
