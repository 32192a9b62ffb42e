#!/bin/bash
# Full GPU suite + smoke, then per-layer forward times and the f9 gradient dump (stops on a fault).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_runs/pytest_gpu.sh "${1:-r4}"
rc=$?
case $rc in 0|1) ;; *) echo "stopping: rc=$rc"; exit $rc;; esac
for L in head down1 down2 down3 nconv4 nconv5 tail; do
  timeout -k 10 60 python3 tools/fwd_layer_bench.py $L 20 2>&1 | tail -1
  r=$?; case $r in 124|134|137|139) exit $r;; esac
done
timeout -k 10 300 python -u tools/f9_dump.py > gpurun_out/f9_dump.log 2>&1
echo "f9_dump rc=$?"
exit $rc
