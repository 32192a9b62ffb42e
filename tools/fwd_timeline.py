#!/usr/bin/env python3
"""The replayed inference forward's kernel timeline from a rocprofv3 kernel trace of
tools/fwd_probe.py (developer tool): steps are delimited by the weight prologue's launch; prints
the last full step's kernels (start, duration in us, queue), the step span and, per kernel name,
the average duration over the last 50 steps.

usage: python3 tools/fwd_timeline.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'weight_prologue' in r['Kernel_Name']]
steps = [(idx[k], idx[k + 1]) for k in range(max(0, len(idx) - 51), len(idx) - 1)]
agg = collections.defaultdict(list)
spans = []
for s, e in steps:
    spans.append((int(rows[e]['Start_Timestamp']) - int(rows[s]['Start_Timestamp'])) / 1e3)
    for r in rows[s:e]:
        agg[r['Kernel_Name'][:110]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
s, e = steps[-1]
t0 = int(rows[s]['Start_Timestamp'])
print(f"step span us: last {spans[-1]:.1f}, mean of {len(spans)} {sum(spans) / len(spans):.1f}")
for r in rows[s:e]:
    st = (int(r['Start_Timestamp']) - t0) / 1e3
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    print(f"{st:8.1f} {d:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:110]}")
print("average per launch:")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {sum(v) / len(v):8.1f} us x{len(v) // max(1, len(steps))} {k}")
