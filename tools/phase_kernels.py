#!/usr/bin/env python3
"""Per-kernel time of the tail of a rocprofv3 kernel trace, from the first launch of a kernel whose
name contains MARKER to the end, divided by N (e.g. the guided training steps of a bench run):
    phase_kernels.py TRACE_CSV MARKER N"""
import collections
import csv
import sys


def main(path, marker, n):
    n = float(n)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    i0 = next(i for i, r in enumerate(rows) if marker in r["Kernel_Name"])
    acc = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows[i0:]:
        k = r["Kernel_Name"]
        k = k[:k.index("(")] if "(" in k else k
        acc[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        cnt[k] += 1
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1000.0
    tot = sum(acc.values())
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1])[:40]:
        print(f"{v / n:9.1f} us  {cnt[k] / n:6.1f} launches  {k[:110]}")
    print(f"kernels {tot / n:.1f} us per step, wall span {span / n:.1f} us per step")


if __name__ == "__main__":
    main(*sys.argv[1:])
