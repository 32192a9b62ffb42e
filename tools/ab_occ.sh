#!/bin/bash
# Occupancy A/B (developer tool): per-layer times and the headline forward for each variant library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/ab_layers.sh "down1 down2 down3 nconv4 nconv5" "$@" > gpurun_out/ab_layers.log 2>&1 || exit $?
for v in cur "$@"; do
  if [ "$v" = cur ]; then lib=""; else lib="$v/libnconv.so"; fi
  out=$(NCONV_LIB=$lib timeout -k 10 120 python3 bench.py --no-train --no-cpu-baseline --no-fp32-forward --no-guided --no-guided-train --steps 100 2>/dev/null | tail -1)
  rc=$?
  echo "$v $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["layer_us"])')" >> gpurun_out/ab_bench.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
cat gpurun_out/ab_layers.log gpurun_out/ab_bench.log
