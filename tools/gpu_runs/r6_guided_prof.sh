#!/bin/bash
# Round 6: kernel statistics of the config-4 guided training step alone (eager driver, 4 steps).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gprof
tag=$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof/p_$tag -o run -- \
    python3 tools/${DRIVER:-guided_train_driver.py} ${REPS:-4} > gpurun_out/gprof/log_$tag.txt 2>&1 || exit $?
f=$(find gpurun_out/gprof/p_$tag -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/gprof/stats_$tag.csv
rm -rf gpurun_out/gprof/p_$tag
python3 - gpurun_out/gprof/stats_$tag.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e6:.2f} ms over the profiled steps (incl. 2 warm-up)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['Percentage']):5.1f}% {int(r['Calls']):5d} {r['Name'][:110]}")
PY
