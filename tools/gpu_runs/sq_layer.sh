#!/bin/bash
# SQ counter passes over one forward layer (tools/fwd_layer_bench.py LAYER 5): usage
#   gpurun -- bash tools/gpu_runs/sq_layer.sh LAYER   -> gpurun_out/sq{A,B}_LAYER/, summary on stdout
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=${1:-head}
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
timeout -k 10 120 python3 tools/fwd_layer_bench.py $L 20 || exit $?
rm -rf gpurun_out/sqA_$L gpurun_out/sqB_$L
timeout -s KILL 90 rocprofv3 --pmc $A --output-format csv -d gpurun_out/sqA_$L -o run -- python3 tools/fwd_layer_bench.py $L 5 > gpurun_out/sqA_$L.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc $B --output-format csv -d gpurun_out/sqB_$L -o run -- python3 tools/fwd_layer_bench.py $L 5 > gpurun_out/sqB_$L.log 2>&1 || exit $?
python3 tools/sq_counters.py gpurun_out/sqA_$L gpurun_out/sqB_$L 100000
