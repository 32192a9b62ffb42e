#!/bin/bash
# Backward kernels after a change: layer-backward tests (every backward arithmetic), per-layer
# backward times per arithmetic and a kernel trace of those runs. Logs in gpurun_out/r3b2_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
stop() { echo "[r3b2] $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -k "backward or accumulate" -m gpu -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r3b2_pytest.log 2>&1 || stop pytest $?
tail -n 2 gpurun_out/r3b2_pytest.log
rm -f gpurun_out/r3b2_layers.log
for m in ${MATHS:-fp32 bf16x3}; do
  for l in nconv2 down1 nconv5 nconv6; do
    NCONV_BWD_MATH=$m timeout -k 10 120 python -u tools/bwd_layer_bench.py $l 20 >> gpurun_out/r3b2_layers.log 2>&1 || stop layer_${m}_$l $?
  done
done
grep bwd gpurun_out/r3b2_layers.log
for m in ${MATHS:-fp32 bf16x3}; do
  NCONV_BWD_MATH=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3b2_prof_$m -o run \
      -- python3 tools/bwd_layer_bench.py ${PROF_LAYER:-nconv2} 10 > gpurun_out/r3b2_prof_$m.log 2>&1 || stop prof_$m $?
  python3 - gpurun_out/r3b2_prof_$m <<'P'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f"{float(r['AverageNs']) / 1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:110]}")
P
done
echo "[r3b2] done"
