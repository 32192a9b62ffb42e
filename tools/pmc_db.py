#!/usr/bin/env python3
"""Summarise rocprofv3 counter passes from their SQLite output (developer tool):
python3 tools/pmc_db.py gpurun_out/pmcA/p_results.db [...] [--kernel SUBSTR]
Prints per kernel (and grid size) the mean per dispatch of every counter collected."""
import collections
import sqlite3
import sys


def main(args):
    sub = None
    if "--kernel" in args:
        i = args.index("--kernel")
        sub = args[i + 1]
        args = args[:i] + args[i + 2:]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in args:
        c = sqlite3.connect(f)
        cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
        rows = c.execute("select * from counters_collection").fetchall()
        for r in rows:
            d = dict(zip(cols, r))
            name = str(d.get("kernel_name", ""))
            if sub and sub not in name:
                continue
            key = (name.split("(")[0][-70:], d.get("grid_size", d.get("grid_size_x", "")))
            agg[key][d["counter_name"]].append(float(d["value"]))
    for (k, g), m in agg.items():
        print(f"{k} grid={g}")
        for cn, v in sorted(m.items()):
            print(f"    {cn:32s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1:])
