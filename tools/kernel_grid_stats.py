#!/usr/bin/env python3
"""Per-(kernel, grid) duration statistics from a rocprofv3 kernel trace.

rocprofv3's kernel_stats.csv averages every dispatch of a kernel symbol; one fwd_tiled
instantiation serves several DNET layers (nconv2 and the three down layers share <8,8,5,PLAIN>)
and the inference forward splits the batch over two streams, so that average mixes grids. This
splits the same trace by grid size, which identifies the launch bench.py times per layer
(time_layers: full batch, one stream).

usage: python3 tools/kernel_grid_stats.py <kernel_trace.csv> <out.csv> [name-filter]
"""
import collections
import csv
import statistics
import sys


def main(src, dst, filt="nconv"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        if filt not in r["Kernel_Name"]:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        agg[(r["Kernel_Name"], grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(dst, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Grid_Size", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs", "MaxNs"])
        for (n, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([n, g, len(v), sum(v), round(sum(v) / len(v), 1), statistics.median(v), min(v), max(v)])
    print(f"wrote {dst}: {len(agg)} (kernel, grid) rows")


if __name__ == "__main__":
    main(*sys.argv[1:])
