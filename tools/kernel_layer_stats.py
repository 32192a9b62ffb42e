#!/usr/bin/env python3
"""Per-layer kernel durations from a rocprofv3 kernel trace of bench.py (developer tool).

bench.time_layers launches each inference kernel of the forward 21 times in a row (1 warm-up +
20 timed, full batch, one stream) in the order below. The MFMA layers share kernel symbols and
persistent grid sizes, so layers are identified by that launch order rather than by name or grid.

usage: python3 tools/kernel_layer_stats.py <kernel_trace.csv> <out.csv>"""
import csv
import statistics
import sys

ORDER = ["nconv1+nconv2_head", "nconv_down1", "nconv_down2", "nconv_down3", "nconv4", "nconv5", "nconv6+7_tail"]
# (without the fused head: "nconv1", "nconv2", ... as separate launches)
ORDER_UNFUSED = ["nconv1", "nconv2"] + ORDER[1:]
RUN = 21


def main(src, dst):
    rows = [r for r in csv.DictReader(open(src)) if "nconv::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    key = lambda r: (r["Kernel_Name"], r["Grid_Size_X"])
    runs, i = [], 0
    while i < len(rows):  # maximal runs of identical consecutive launches
        j = i
        while j < len(rows) and key(rows[j]) == key(rows[i]):
            j += 1
        runs.append(rows[i:j])
        i = j
    # the time_layers block: the last len(ORDER) runs of length >= RUN (a run may merge two
    # layers with the same symbol and grid: split those into RUN-long pieces)
    pieces = []
    for r in runs:
        if len(r) >= RUN:
            pieces += [r[k:k + RUN] for k in range(0, len(r) - RUN + 1, RUN)]
    order = ORDER_UNFUSED if any("fwd_tiled<1, 8, 5, 1" in p[0]["Kernel_Name"] for p in pieces[-len(ORDER_UNFUSED):]) \
        else ORDER
    pieces = pieces[-len(order):]
    with open(dst, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Layer", "Kernel_Name", "Grid_Size", "Calls", "AverageNs", "MedianNs", "MinNs", "MaxNs"])
        for name, p in zip(order, pieces):
            d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in p[1:]]  # skip the warm-up
            w.writerow([name, p[0]["Kernel_Name"][:120], p[0]["Grid_Size_X"], len(d), round(sum(d) / len(d), 1),
                        statistics.median(d), min(d), max(d)])
            print(f"{name:16s} {sum(d) / len(d) / 1e3:8.2f} us  {p[0]['Kernel_Name'][:70]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
