#!/usr/bin/env python3
"""Kernel-time breakdown of the last N iterations of a rocprofv3 kernel trace (developer tool).

usage: python3 tools/prof_last.py <trace dir> <marker substring> <markers per iteration> <iterations>
Iterations are delimited by launches of the marker kernel (e.g. 'fwd_tiled<1, 8, 5, 1').
"""
import collections
import csv
import glob
import sys


def main(d, marker, per_it, n_it):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                   for r in csv.DictReader(open(f))), key=lambda r: r[1])
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    sel = rows[idx[-per_it * n_it]:]
    agg = collections.defaultdict(list)
    for n, s, e in sel:
        agg[n].append(e - s)
    tot = sum(sum(v) for v in agg.values())
    span = (sel[-1][2] - sel[0][1]) / 1e6
    print(f"kernel time {tot / n_it / 1e6:.3f} ms/iter, span {span / n_it:.3f} ms/iter")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:30]:
        print(f"{sum(v) / tot * 100:5.1f}% {sum(v) / n_it / 1e6:7.3f} ms/it n/it={len(v) / n_it:5.1f} "
              f"avg {sum(v) / len(v) / 1e3:8.1f} us {n[:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
