#!/usr/bin/env python3
"""Per-kernel time of one training step from a rocprofv3 kernel trace of bench.py: kernels whose
launch count is a multiple of the training step count, grouped by (kernel, grid), in us per step.
Usage: train_kernels.py TRACE_CSV STEPS_PER_RUN"""
import collections
import csv
import sys


def main(path, calls):
    calls = int(calls)
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
        acc[(r["Kernel_Name"], g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for (k, g), v in acc.items():
        if len(v) % calls == 0 and len(v) // calls <= 4:
            rows.append((sum(v) / calls / 1000.0, len(v) // calls, k, g))
    rows.sort(reverse=True)
    tot = 0.0
    for us, n, k, g in rows:
        tot += us
        print(f"{us:8.1f} us  x{n}  grid {g:>8}  {k[:100]}")
    print(f"total {tot:.1f} us per step (kernels with call count a multiple of {calls})")


if __name__ == "__main__":
    main(*sys.argv[1:])
