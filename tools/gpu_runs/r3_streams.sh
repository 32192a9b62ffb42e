#!/bin/bash
# Forward parity after a forward-kernel change, then the config-2 bench at several stream splits.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { echo "[r3s] $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py -m gpu -q \
   --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r3s_pytest.log 2>&1 || stop pytest $?
tail -1 gpurun_out/r3s_pytest.log
for cfg in "1 1" "2 1" "1 2" "4 1" "2 2" "1 1"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-train --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline \
     --steps 30 --warmup 5 --inference-streams $1 --mid-streams $2 > gpurun_out/r3s_bench.log 2>&1 || stop bench $?
  python3 -c "import json; d=json.loads(open('gpurun_out/r3s_bench.log').read().strip().splitlines()[-1]); print('streams $1 mid $2', d['value'], d['ms_per_step'])"
done
python3 -c "import json; d=json.loads(open('gpurun_out/r3s_bench.log').read().strip().splitlines()[-1]); print(json.dumps(d['layer_us']))"
