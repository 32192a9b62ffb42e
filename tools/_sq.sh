#!/bin/bash
# SQ counter passes over single-layer exact-fp32 forwards (developer probe).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export NCONV_FWD_MATH=fp32
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
C="SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FMA_F32 SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM_NORM SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE"
for L in ${LAYERS:-nconv2 down1}; do
  timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 20 || exit $?
  for P in A B C; do
    timeout -s KILL 60 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sq${P}_$L -o run -- python3 tools/fwd_layer_bench.py $L 5 > gpurun_out/sq${P}_$L.log 2>&1 || { echo "pass $P $L failed"; tail -5 gpurun_out/sq${P}_$L.log; }
  done
done
echo done
