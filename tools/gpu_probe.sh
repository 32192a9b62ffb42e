#!/bin/bash
# Development GPU probe: GPU test suite, then SQ counter passes over single-layer forward runs.
# Stops at the first step that times out / aborts / faults (exit 124, 134, 137, 139).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  echo "[probe] $name" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[probe] $name rc=$rc" >&2
  tail -3 "gpurun_out/$name.log" >&2
  if fatal $rc; then exit $rc; fi
  return 0
}
if [ "${PROBE_TESTS:-1}" = 1 ]; then
  step pytest_gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
for L in ${PROBE_LAYERS:-head down1 tail}; do
  step time_$L 60 python3 tools/fwd_layer_bench.py $L 20
done
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
if [ "${PROBE_PMC:-1}" = 1 ]; then
  for L in ${PROBE_LAYERS:-head down1 tail}; do
    step pmcA_$L 60 rocprofv3 --pmc $A --output-format csv -d gpurun_out/pmcA_$L -o run -- python3 tools/fwd_layer_bench.py $L 5
    step pmcB_$L 60 rocprofv3 --pmc $B --output-format csv -d gpurun_out/pmcB_$L -o run -- python3 tools/fwd_layer_bench.py $L 5
  done
fi
echo "[probe] done" >&2
