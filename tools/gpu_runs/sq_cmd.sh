#!/bin/bash
# SQ counter passes over an arbitrary short GPU command: gpurun -- bash tools/gpu_runs/sq_cmd.sh TAG MIN_GRID CMD...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=$1; G=$2; shift 2
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
rm -rf gpurun_out/sqA_$T gpurun_out/sqB_$T
timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d gpurun_out/sqA_$T -o run -- "$@" > gpurun_out/sqA_$T.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $B --output-format csv -d gpurun_out/sqB_$T -o run -- "$@" > gpurun_out/sqB_$T.log 2>&1 || exit $?
python3 tools/sq_counters.py gpurun_out/sqA_$T gpurun_out/sqB_$T $G
