#!/bin/bash
# Backward probe: layer backward tests, per-layer backward timing for each weight-gradient math,
# and SQ counters of the bf16 weight gradient on nconv2.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_layers.py -k backward -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_bwd.log 2>&1
rc=$?; echo "pytest layers rc=$rc"; grep -E "g_w \[bf|passed|failed" gpurun_out/pytest_bwd.log | tail -24
case $rc in 124|134|137|139) exit $rc;; esac
for L in nconv2 nconv6; do for M in fp32 bf16x3; do
  NCONV_BWD_MATH=$M timeout -k 10 60 python3 tools/bwd_layer_bench.py $L 10 || exit $?
done; done
for L in nconv2 nconv6; do
  NCONV_BWD_MATH=bf16x3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ktbw_$L -o run -- python3 tools/bwd_layer_bench.py $L 5 > gpurun_out/ktbw_$L.log 2>&1 || exit $?
done
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for P in A B; do
  NCONV_BWD_MATH=bf16x3 timeout -s KILL 60 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sqbw${P} -o run -- python3 tools/bwd_layer_bench.py nconv2 3 > gpurun_out/sqbw${P}.log 2>&1 || echo "pmc $P failed"
done
echo done
