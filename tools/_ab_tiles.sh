#!/bin/bash
# A/B of the exact-fp32 forward's output-channel slices (NCONV_TILED_CS; 0 = by layer size).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cs in ${CFGS:-1 0 2 4}; do
  NCONV_TILED_CS=$cs timeout -k 10 200 python -u bench.py --math fp32 --alt-math '' --no-config5 --no-train --no-guided --no-guided-train --no-cpu-baseline --steps 40 > gpurun_out/ab_cs_$cs.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_cs_$cs.log').read().strip().splitlines()[-1]); print('$cs', d['ms_per_step'], d['layer_us'])"
done
if [ "${TESTS:-0}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_golden.py tests/test_gpu_dnet.py tests/test_gpu_train_graph.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_tiles.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_tiles.log
exit $rc
fi
