#!/bin/bash
# Phase path check: its parity tests + the DNET / golden tests, then layer times with and without
# phase weights, then the config-2 bench line. Logs: gpurun_out/r3phase_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { echo "[r3phase] $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py -m gpu -q \
   --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r3phase_pytest.log 2>&1 || stop pytest $?
tail -2 gpurun_out/r3phase_pytest.log
for ph in 0 1 0 1; do
  for l in nconv5 nconv4 tail; do
    NCONV_PHASE=$ph timeout -k 10 120 python -u tools/fwd_layer_bench.py $l 30 2>/dev/null | sed "s/^/phase=$ph /" || stop layer $?
  done
done
timeout -k 10 300 python -u bench.py --no-train --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline \
   --steps 30 --warmup 5 > gpurun_out/r3phase_bench.log 2>&1 || stop bench $?
python3 -c "import json; d=json.loads(open('gpurun_out/r3phase_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['layer_us']))"
