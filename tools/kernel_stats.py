#!/usr/bin/env python3
"""Per-kernel time summary from a rocprofv3 --kernel-trace database or kernel_stats.csv
(developer tool): python3 tools/kernel_stats.py <dir-or-file> [top]"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def rows_from(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        csvs = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = (dbs or csvs)[0]
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        name = "kernel_name" if "kernel_name" in cols else "name"
        for n, s, e in c.execute(f"select {name}, start, end from kernels"):
            yield n, e - s
    else:
        for r in csv.DictReader(open(path)):
            yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main(path, top):
    agg = collections.defaultdict(list)
    for n, d in rows_from(path):
        agg[n].append(d)
    tot = sum(sum(v) for v in agg.values())
    print(f"total kernel time {tot/1e6:.3f} ms over {sum(len(v) for v in agg.values())} dispatches")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print(f"{sum(v)/tot*100:5.1f}%  {sum(v)/1e6:8.3f} ms  n={len(v):5d}  avg {sum(v)/len(v)/1e3:9.2f} us  {n[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
