#!/bin/bash
# Round 6: SQ counter passes over the eager config-2 training step (tools/train_probe.py --eager),
# one rocprofv3 --pmc run per pass under its own limit; per-kernel summary via tools/sq_counters.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sqt
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
C="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
timeout -k 10 120 python3 tools/train_probe.py --eager --steps 3 > gpurun_out/sqt/time.log 2>&1 || exit $?
tail -n 1 gpurun_out/sqt/time.log
for P in A B C; do
  timeout -k 10 120 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sqt/pmc$P -o run -- \
      python3 tools/train_probe.py --eager --steps 2 > gpurun_out/sqt/pmc$P.log 2>&1 || exit $?
done
python3 tools/sq_counters.py gpurun_out/sqt/pmcA gpurun_out/sqt/pmcB 1000 > gpurun_out/sqt/sum.txt
python3 tools/sq_counters.py gpurun_out/sqt/pmcC gpurun_out/sqt/pmcC 1000 >> gpurun_out/sqt/sum.txt
grep -E "wgrad|dgrad" gpurun_out/sqt/sum.txt | cut -c1-330
