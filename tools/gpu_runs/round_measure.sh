#!/bin/bash
# End-of-milestone GPU measurement (run through gpurun): GPU tests, smoke, bench line, rocprofv3
# kernel-trace/stats of the same bench command, PMC HBM-traffic passes. Outputs in gpurun_out/.
# Stops at the first step that times out / aborts / faults (exit 124, 134, 137, 139) or fails.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  echo "[measure] $name" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[measure] $name rc=$rc" >&2
  tail -2 "gpurun_out/$name.log" >&2
  [ $rc -eq 0 ] || exit $rc
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python -u bench.py
cp gpurun_out/bench.log gpurun_out/bench.json
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/pmc_traffic.py run
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/pmc_traffic.py run
echo "[measure] done" >&2
