#!/bin/bash
# Backward change check: layer / phase / accumulate backward tests, DNET and golden training
# gradients, the training-step bench leg and per-layer backward times. Logs in gpurun_out/r3b3_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { echo "[r3b3] $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_dnet.py tests/test_gpu_golden.py \
    -k "backward or accumulate or train or f1_layer or f3" -m gpu -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r3b3_pytest.log 2>&1 || stop pytest $?
tail -n 2 gpurun_out/r3b3_pytest.log
timeout -k 10 300 python -u bench.py --math fp32 --alt-math '' --no-config5 --no-guided --no-guided-train \
    --no-cpu-baseline --steps 30 > gpurun_out/r3b3_bench.log 2>&1 || stop bench $?
python3 -c "import json; d=json.loads(open('gpurun_out/r3b3_bench.log').read().strip().splitlines()[-1]); t=d['train_fwd_bwd_adamw']; print('fwd', d['value'], d['ms_per_step'], 'train', t.get('ms_per_step'), t.get('frames_per_sec'))"
rm -f gpurun_out/r3b3_layers.log
for l in nconv2 down1 nconv5 nconv6; do
  timeout -k 10 120 python -u tools/bwd_layer_bench.py $l 20 >> gpurun_out/r3b3_layers.log 2>&1 || stop layer_$l $?
done
grep bwd gpurun_out/r3b3_layers.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3b3_prof -o run \
    -- python3 bench.py --math fp32 --alt-math '' --no-config5 --no-guided --no-guided-train --no-cpu-baseline --steps 10 \
    > gpurun_out/r3b3_prof.log 2>&1 || stop prof $?
python3 - gpurun_out/r3b3_prof <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(f"{float(r['AverageNs']) / 1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:110]}")
P
echo "[r3b3] done"
