import csv, sys
from collections import defaultdict
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
ad = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name']]
# last full step: between the last two adamw kernels
a, b = ad[-2], ad[-1]
step = rows[a + 1: b + 1]
t0 = int(step[0]['Start_Timestamp']); t1 = int(step[-1]['End_Timestamp'])
print(f"step wall (first kernel start -> adamw end): {(t1 - t0) / 1e3:.1f} us, kernels {len(step)}")
by_q = defaultdict(float)
for r in step:
    by_q[r['Queue_Id'] + '/' + r['Stream_Id']] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
print("busy per queue/stream (us):", dict(by_q))
# union of busy intervals
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in step)
busy = 0; cs, ce = iv[0]
for s, e in iv[1:]:
    if s > ce:
        busy += ce - cs; cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"GPU busy (union): {busy / 1e3:.1f} us, idle gaps: {(t1 - t0 - busy) / 1e3:.1f} us")
# group by phase: forward until first 'xent', backward until adamw
agg = defaultdict(float)
for r in step:
    n = r['Kernel_Name']
    key = n.split('(')[0].replace('void ', '')[:60]
    agg[key] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v:9.1f} us  {k}")
