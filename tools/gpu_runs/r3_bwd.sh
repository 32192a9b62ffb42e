#!/bin/bash
# Round 3: backward arithmetic on hardware. Layer-backward tests (with the nconv_plan assertion),
# the training-step bench leg and per-layer backward times under each bwd_math, a rocprofv3 kernel
# trace of the bf16x3 training step, and the export probe. Logs in gpurun_out/r3bwd_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { echo "[r3bwd] $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -k "backward or accumulate" -m gpu -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r3bwd_pytest.log 2>&1 || stop pytest $?
tail -2 gpurun_out/r3bwd_pytest.log
for m in fp32 bf16x3 bf16x9; do
  NCONV_BWD_MATH=$m timeout -k 10 300 python -u bench.py --math fp32 --alt-math '' --no-config5 --no-guided \
      --no-guided-train --no-cpu-baseline --steps 20 > gpurun_out/r3bwd_bench_$m.log 2>&1 || stop bench_$m $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r3bwd_bench_$m.log').read().strip().splitlines()[-1]); t=d['train_fwd_bwd_adamw']; print('$m', t.get('ms_per_step'), t.get('value'))"
  for l in nconv2 down1 nconv5 nconv6; do
    NCONV_BWD_MATH=$m timeout -k 10 120 python -u tools/bwd_layer_bench.py $l 20 >> gpurun_out/r3bwd_layers.log 2>&1 || stop layer_$m_$l $?
  done
done
cat gpurun_out/r3bwd_layers.log
NCONV_BWD_MATH=bf16x3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3bwd_prof -o run \
    -- python3 bench.py --math fp32 --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline --steps 10 \
    > gpurun_out/r3bwd_prof.log 2>&1 || stop prof $?
timeout -k 10 300 python -u tools/export_probe.py > gpurun_out/r3_export_probe.log 2>&1 || stop export_probe $?
cat gpurun_out/r3_export_probe.log
MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 timeout -k 10 300 python -u tools/export_probe.py > gpurun_out/r3_export_probe_miopen.log 2>&1 || stop export_probe_log $?
echo "[r3bwd] done"
