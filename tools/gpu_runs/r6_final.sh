#!/bin/bash
# Round-6 measurement: full GPU suite + smoke, bench line, rocprofv3 kernel trace/stats of the bench,
# PMC HBM-traffic passes, SQ counter passes of the head at 5 % and 40 % density and of the one-kernel
# backward. Stops at the first step that times out / aborts / faults.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sq
tag=${1:-r6}
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  echo "[measure] $name" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[measure] $name rc=$rc" >&2
  tail -3 "gpurun_out/$name.log" >&2
  case $rc in 0) ;; 1) [ "$name" = "pytest_$tag" ] || exit 1;; *) exit $rc;; esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_$tag 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
  step smoke_$tag 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_$tag 600 python3 -u bench.py
cp gpurun_out/bench_$tag.log gpurun_out/bench_$tag.json
step prof_$tag 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu-baseline
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/pmc_traffic.py run
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/pmc_traffic.py run
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
C="SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"
for D in 0.05 0.40; do
  export NCONV_DENSITY=$D
  for P in A C; do
    step sq_head_${D}_$P 60 rocprofv3 --pmc ${!P} --output-format csv -d gpurun_out/sq/pmc${P}_head_$D -o run -- python3 tools/fwd_layer_bench.py head 5
  done
done
echo "[measure] done" >&2
