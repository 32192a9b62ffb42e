#!/bin/bash
# Small channel-split layers (fwd_tiled, two output channels per thread) with their kernel rows
# unrolled so a plane's weight loads issue up front (variants/us) vs the in-tree library:
# forward parity tests on the variant, then the forward bench alternated (per-layer times).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/us
NCONV_LIB=$PWD/variants/us/libnconv.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 \
    --timeout-method thread -m gpu tests/test_gpu_dnet.py tests/test_gpu_golden.py tests/test_gpu_layers.py \
    > gpurun_out/us/pytest.log 2>&1
rc=$?; echo "us: $(tail -1 gpurun_out/us/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for V in base us; do
    lib=""; [ $V != base ] && lib=$PWD/variants/$V/libnconv.so
    NCONV_LIB=$lib timeout -k 10 200 python3 bench.py --no-train --no-config5 --no-guided \
        --no-guided-train --no-cpu-baseline --alt-math "" --head-density 0 > gpurun_out/us/bench_${V}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], d['value'], ' '.join(f'{k}={v}' for k,v in d['layer_us'].items()))" gpurun_out/us/bench_${V}_$rep.json $V
  done
done
