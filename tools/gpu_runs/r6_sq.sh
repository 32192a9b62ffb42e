#!/bin/bash
# Round 6: per-layer forward times and SQ counter passes (one rocprofv3 --pmc run per pass, each
# under its own limit) for the layers named in $FWD (tools/fwd_layer_bench.py names).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sq6
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/sq6/$name.log" 2>&1
  local rc=$?
  echo "[probe] $name rc=$rc $(tail -1 gpurun_out/sq6/$name.log)"
  if fatal $rc; then exit $rc; fi
  return 0
}
FWD=${FWD:-tail tailc}
for L in $FWD; do step time_$L 60 python3 tools/fwd_layer_bench.py $L 20; done
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
C="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
for L in $FWD; do
  for P in A B C; do
    step pmc${P}_$L 60 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sq6/pmc${P}_$L -o run -- python3 tools/fwd_layer_bench.py $L 5
  done
  python3 tools/sq_counters.py gpurun_out/sq6/pmcA_$L gpurun_out/sq6/pmcB_$L 1000 > gpurun_out/sq6/sum_$L.txt
  python3 tools/sq_counters.py gpurun_out/sq6/pmcC_$L gpurun_out/sq6/pmcC_$L 1000 >> gpurun_out/sq6/sum_$L.txt
  cat gpurun_out/sq6/sum_$L.txt
done
