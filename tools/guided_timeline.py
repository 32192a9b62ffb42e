#!/usr/bin/env python3
"""Per-queue summary of one config-4 guided training step from a rocprofv3 kernel trace of
tools/guided_train_driver.py (developer tool): steps are delimited by step 1's weight prologue;
prints, for the last full step, each queue's busy time, first start and last end, and the 25
longest kernels with their queue.

usage: python3 tools/guided_timeline.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "prologue" in r["Kernel_Name"] or "weight_prep" in r["Kernel_Name"]]
s, e = idx[-2], idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
print("step span us", (int(rows[e]["Start_Timestamp"]) - t0) / 1e3, "kernels", e - s)
q = collections.defaultdict(lambda: [0.0, 1e18, 0.0, 0])
for r in rows[s:e]:
    a, b = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    v = q[r["Queue_Id"]]
    v[0] += b - a
    v[1] = min(v[1], a)
    v[2] = max(v[2], b)
    v[3] += 1
for k, (busy, first, last, n) in sorted(q.items()):
    print(f"queue {k}: {n} kernels, busy {busy:.0f} us, {first:.0f} .. {last:.0f} us")
print("longest:")
for r in sorted(rows[s:e], key=lambda r: int(r["Start_Timestamp"]) - int(r["End_Timestamp"]))[:25]:
    a = (int(r["Start_Timestamp"]) - t0) / 1e3
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{a:9.1f} {d:8.1f} q{r['Queue_Id']} {r['Kernel_Name'][:90]}")
