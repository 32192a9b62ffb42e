#!/bin/bash
# fwd_tiled timing probes (wrong results; per-layer times only): variants/pw = weights as
# constants (no scalar loads), variants/pl = each staged plane read from LDS once per plane
# instead of once per kernel row; against variants/base.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tp
for rep in 1 2; do
  for V in base pw pl; do
    NCONV_LIB=$PWD/variants/$V/libnconv.so timeout -k 10 200 python3 bench.py --no-train --no-config5 --no-guided \
        --no-guided-train --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/tp/bench_${V}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], d['value'], ' '.join(f'{k}={v}' for k,v in d['layer_us'].items()))" gpurun_out/tp/bench_${V}_$rep.json $V
  done
done
