#!/usr/bin/env python3
"""One training step's kernel timeline from a rocprofv3 kernel trace of tools/train_probe.py
(developer tool): steps are delimited by the weight prologue's launch (weight_prep, or
train_prologue from round 5); prints the last full step's
kernels (start, duration in us, queue) and the sum of their durations.

usage: python3 tools/step_timeline.py <run_kernel_trace.csv>"""
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'weight_prep' in r['Kernel_Name'] or 'train_prologue' in r['Kernel_Name']]
# average per-kernel durations over steps 5..end, and print one step timeline
steps=[(idx[k],idx[k+1]) for k in range(5,len(idx)-1)]
agg=collections.defaultdict(list)
for s,e in steps:
    cnt=collections.Counter()
    for r in rows[s:e]:
        n=r['Kernel_Name'][:95]; cnt[n]+=1
        agg[(n,cnt[n])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
s,e=steps[-1]
t0=int(rows[s]['Start_Timestamp'])
print('step span us', (int(rows[e]['Start_Timestamp'])-t0)/1e3)
tot=0
for r in rows[s:e]:
    st=(int(r['Start_Timestamp'])-t0)/1e3; d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3; tot+=d
    print(f"{st:8.1f} {d:7.1f} q{r['Queue_Id']} {r['Kernel_Name'][:95]}")
print('sum of kernel durations', tot)
small=[r for r in rows[s:e] if (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 < 8.0]
print('kernels under 8 us:', len(small), 'of', e-s)
