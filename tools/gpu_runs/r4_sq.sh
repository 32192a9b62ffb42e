#!/bin/bash
# Round-4 counter probe: available counters, per-layer forward / backward times, and SQ counter
# passes (one rocprofv3 --pmc run per pass, each under its own time limit) for the exact-fp32
# forward kernels and nconv2's backward. Stops at the first step that times out / aborts / faults.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sq
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  echo "[probe] $name" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/sq/$name.log" 2>&1
  local rc=$?
  echo "[probe] $name rc=$rc" >&2
  tail -2 "gpurun_out/sq/$name.log" >&2
  if fatal $rc; then exit $rc; fi
  return 0
}
step avail 60 rocprofv3 --list-avail
FWD=${FWD_LAYERS:-head down1 down2 down3 nconv4 nconv5 tail}
BWD=${BWD_LAYERS:-nconv2 nconv6}
for L in $FWD; do step time_$L 60 python3 tools/fwd_layer_bench.py $L 20; done
for L in $BWD; do step btime_$L 60 python3 tools/bwd_layer_bench.py $L 10; done
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
C="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
for L in $FWD; do
  for P in A B C; do
    step pmc${P}_$L 60 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sq/pmc${P}_$L -o run -- python3 tools/fwd_layer_bench.py $L 5
  done
done
for L in $BWD; do
  for P in A B C; do
    step bpmc${P}_$L 90 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sq/bpmc${P}_$L -o run -- python3 tools/bwd_layer_bench.py $L 3
  done
done
echo "[probe] done" >&2
