#!/bin/bash
# Training-path tests after a forward change, the bench line with the training leg, and the two
# PMC passes (FETCH_SIZE, WRITE_SIZE) of tools/pmc_traffic.py. Logs: gpurun_out/r3tp_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { echo "[r3tp] $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_dnet.py tests/test_gpu_train_graph.py \
   tests/test_gpu_loss.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf \
   > gpurun_out/r3tp_pytest.log 2>&1 || stop pytest $?
tail -1 gpurun_out/r3tp_pytest.log
timeout -k 10 400 python -u bench.py --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline --steps 20 \
   > gpurun_out/r3tp_bench.log 2>&1 || stop bench $?
python3 -c "import json; d=json.loads(open('gpurun_out/r3tp_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['layer_us'])); t=d['train_fwd_bwd_adamw']; print('train', t['ms_per_step'], t['frames_per_sec'])"
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/pmc_traffic.py run \
   > gpurun_out/r3tp_pmc_fetch.log 2>&1 || stop pmc_fetch $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/pmc_traffic.py run \
   > gpurun_out/r3tp_pmc_write.log 2>&1 || stop pmc_write $?
echo "[r3tp] done"
