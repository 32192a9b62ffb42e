#!/bin/bash
# Same-box A/B of forward-kernel variants (variants/<name>/libnconv.so via NCONV_LIB) against the
# in-tree library: single-layer times alternated, outputs compared bitwise, forward-only bench lines.
# Usage: r5_fwd_ab.sh "layer ..." variant ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fwdab
layers=$1; shift
for rep in 1 2; do
  for L in $layers; do
    b=$(timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 50 2>/dev/null | tail -1); r=$?
    case $r in 0) ;; *) echo "base $L rc=$r"; exit $r;; esac
    line="base $b"
    for V in "$@"; do
      c=$(NCONV_LIB=$PWD/variants/$V/libnconv.so timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 50 2>/dev/null | tail -1); r=$?
      case $r in 0) ;; *) echo "$V $L rc=$r"; exit $r;; esac
      line="$line | $V $c"
    done
    echo "$line"
  done
done
timeout -k 10 120 python3 tools/fwd_out_dump.py gpurun_out/fwdab/base.pt > /dev/null 2>&1 || exit 1
for V in "$@"; do
  NCONV_LIB=$PWD/variants/$V/libnconv.so timeout -k 10 120 python3 tools/fwd_out_dump.py gpurun_out/fwdab/$V.pt > /dev/null 2>&1 || exit 1
  python3 -c "import torch,sys; a=torch.load(sys.argv[1]); b=torch.load(sys.argv[2]); print(sys.argv[3], 'bitwise' if torch.equal(a,b) else 'DIFFERENT max %.3e' % (a-b).abs().max().item())" gpurun_out/fwdab/base.pt gpurun_out/fwdab/$V.pt $V
done
for V in base "$@"; do
  lib=""; [ "$V" != base ] && lib=$PWD/variants/$V/libnconv.so
  NCONV_LIB=$lib timeout -k 10 200 python3 bench.py --no-train --no-config5 --no-guided --no-guided-train \
      --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/fwdab/bench_$V.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['layer_us'])" gpurun_out/fwdab/bench_$V.json $V
done
