#!/bin/bash
# Round 6 iteration: selected GPU tests (-s, every failure listed), then the bench.
#   gpurun --timeout 900 -- bash tools/gpu_runs/r6_iter.sh TAG "tests/test_a.py tests/test_b.py" [bench args]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-iter}; tests=${2:-tests}; shift 2; bargs="$*"
timeout -k 10 600 python -u -m pytest $tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -rf \
    > gpurun_out/iter_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/iter_$tag.log | tail -15
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u bench.py $bargs > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bench_$tag.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step']); print('layers', d.get('layer_us')); r=d['roofline']; print('roof', r['kernel'], r['kernel_us'], r['frac'], r.get('replayed_shape'))
t=d.get('train_fwd_bwd_adamw'); print('train', t and t['ms_per_step']); g=d.get('guided_fwd'); print('guided', g and g['fp32_mfma_frac']); gt=d.get('guided_train_fwd_bwd_adamw'); print('gtrain', gt and gt['ms_per_step'])
"
exit $rc
