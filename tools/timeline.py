"""Concurrency timeline of one training step from a rocprofv3 kernel trace of bench.py.

Picks step `--step i` (default: the 6th embedding sort .. the 7th, i.e. inside the timed region of
`bench.py --warmup 3`), then reports how long 0 / 1 / 2 / 3 / 4+ kernels run at once, and lists the
serial stretches (exactly one kernel active for more than `--min-us`), which are the step's critical
chain segments with nothing beside them.
Usage: python tools/timeline.py <rocprof dir> [--step i] [--min-us 5]"""
import csv
import sys
from collections import defaultdict

d = sys.argv[1]
step_i = int(sys.argv[sys.argv.index("--step") + 1]) if "--step" in sys.argv else 5
min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 5.0
rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "embed_sort" in r["Kernel_Name"]]
a, b = st[step_i], st[step_i + 1]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in step)
short = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ergm::", "")[:70]  # noqa: E731
ev = []
for k, r in enumerate(step):
    ev.append((int(r["Start_Timestamp"]), 1, k))
    ev.append((int(r["End_Timestamp"]), -1, k))
ev.sort()
active = set()
hist = defaultdict(float)
serial = []
prev = t0
for t, kind, k in ev:
    if t > prev:
        n = len(active)
        hist[min(n, 4)] += (t - prev) / 1e3
        if n == 1:
            (only,) = tuple(active)
            serial.append((prev, t, only))
    prev = t
    if kind == 1:
        active.add(k)
    else:
        active.discard(k)
print(f"step {step_i}: wall {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
print("time with n kernels active (us): " + "  ".join(f"{n}:{hist[n]:.1f}" for n in range(5)))
# merge consecutive serial slices of the same kernel
merged = []
for s, e, k in serial:
    if merged and merged[-1][2] == k and s - merged[-1][1] < 1000:
        merged[-1] = (merged[-1][0], e, k)
    else:
        merged.append((s, e, k))
by_k = defaultdict(float)
for s, e, k in merged:
    by_k[short(step[k])] += (e - s) / 1e3
print("serial time by kernel (only kernel running):")
for n, v in sorted(by_k.items(), key=lambda kv: -kv[1])[:25]:
    print(f"  {v:8.1f} us  {n}")
print(f"serial stretches > {min_us} us:")
for s, e, k in merged:
    if (e - s) / 1e3 > min_us:
        print(f"  t={(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f} us  {short(step[k])}")
