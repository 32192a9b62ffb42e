#!/bin/bash
# A/B of forward-kernel variants (libnconv builds under _exp/<name>/, tools/build_variant.sh):
#   gpurun -- bash tools/gpu_runs/ab_fwd.sh "r0p0 r1p1" [TESTVARIANT]
# Per variant: every exact-fp32 layer's time (tools/fwd_layer_bench.py) and the config-2 forward
# bench line; TESTVARIANT (optional) first runs the forward layer + DNET parity tests on it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/ab_fwd.log; : > $out
stop() { echo "[ab] $1 rc=$2" | tee -a $out; exit $2; }
if [ -n "$2" ]; then
  NCONV_LIB=_exp/$2/libnconv.so timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_dnet.py \
     tests/test_gpu_golden.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf \
     > gpurun_out/ab_fwd_pytest.log 2>&1 || stop pytest $?
  tail -1 gpurun_out/ab_fwd_pytest.log | tee -a $out
fi
for v in $1; do
  for l in ${LAYERS:-nconv1 nconv2 down1 down2 down3 nconv4 nconv5 tail}; do
    NCONV_LIB=_exp/$v/libnconv.so timeout -k 10 120 python -u tools/fwd_layer_bench.py $l 30 2>/dev/null | sed "s/^/$v /" >> $out || stop $v-$l $?
  done
  NCONV_LIB=_exp/$v/libnconv.so timeout -k 10 300 python -u bench.py --no-train --alt-math '' --no-config5 --no-guided \
     --no-guided-train --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/ab_fwd_bench_$v.log 2>&1 || stop bench-$v $?
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_fwd_bench_$v.log').read().strip().splitlines()[-1]); print('$v bench', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))" >> $out
done
cat $out
