#!/bin/bash
# Forward-kernel change check: layer / DNET / golden / export GPU tests, then the config-2 bench line
# (headline only) twice. Logs: gpurun_out/r3fc_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { echo "[r3fc] $1 rc=$2"; exit $2; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py \
   tests/test_export.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf \
   > gpurun_out/r3fc_pytest.log 2>&1 || stop pytest $?
tail -1 gpurun_out/r3fc_pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-train --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline \
     --steps 30 --warmup 5 ${BENCH_ARGS} > gpurun_out/r3fc_bench.log 2>&1 || stop bench $?
  python3 -c "import json; d=json.loads(open('gpurun_out/r3fc_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['layer_us']))"
done
for l in tail nconv5; do
  timeout -k 10 120 python -u tools/fwd_layer_bench.py $l 50 || stop layer_$l $?
done
