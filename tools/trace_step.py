"""Per-step breakdown of a rocprofv3 kernel trace of bench.py: the last complete training step
(embedding sort of step i .. embedding sort of step i+1), busy time per stream, idle gaps and
the top kernels.  Usage: python tools/trace_step.py <rocprof output dir> [top-N]"""
import csv, sys
from collections import defaultdict
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
st = [i for i, r in enumerate(rows) if 'embed_sort' in r['Kernel_Name']]
a, b = st[-2], st[-1]
step = rows[a:b]
t0 = int(step[0]['Start_Timestamp']); t1 = max(int(r['End_Timestamp']) for r in step)
print(f"step wall (embedding forward -> last kernel end): {(t1 - t0) / 1e3:.1f} us, kernels {len(step)}")
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
cnt = defaultdict(int)
for r in step:
    cnt[r['Kernel_Name'].split('(')[0].replace('void ', '')[:60]] += 1
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{v:9.1f} us  x{cnt[k]:<4d} {k}")
# main-stream idle gaps > 8 us (what the critical path waits for)
if "--gaps" in sys.argv:
    main_q = max(by_q, key=by_q.get)
    ms = [r for r in step if r['Queue_Id'] + '/' + r['Stream_Id'] == main_q]
    short = lambda r: r['Kernel_Name'].split('(')[0].replace('void ', '').replace('ergm::', '')[:48]  # noqa: E731
    for p, q in zip(ms, ms[1:]):
        g = (int(q['Start_Timestamp']) - int(p['End_Timestamp'])) / 1e3
        if g > 8:
            print(f"gap {g:7.1f} us at t={(int(p['End_Timestamp']) - t0) / 1e3:8.1f}: {short(p)} -> {short(q)}")
# main-stream time by phase and kernel class
if "--phases" in sys.argv:
    main_q = max(by_q, key=by_q.get)
    ph, cur = defaultdict(lambda: defaultdict(float)), "forward"
    for r in step:
        n = r['Kernel_Name']
        if 'xent_kernel' in n:
            cur = "loss+head bwd"
        elif 'attn_bwd' in n and cur == "loss+head bwd":
            cur = "layers bwd"
        elif 'embed_runsum' in n:
            cur = "embed bwd"
        q = r['Queue_Id'] + '/' + r['Stream_Id']
        cls = ('gemm' if 'gemm' in n or 'splitk' in n else 'attn' if 'attn' in n else
               'ln' if 'ln_' in n else 'adamw' if 'adamw' in n else 'other')
        ph[(cur, 'main' if q == main_q else 'side')][cls] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    for k, v in ph.items():
        print(f"{k[0]:14s} {k[1]:5s} total {sum(v.values()):8.1f} us  " +
              "  ".join(f"{c}={t:.0f}" for c, t in sorted(v.items(), key=lambda kv: -kv[1])))
if "--gapstats" in sys.argv:
    main_q = max(by_q, key=by_q.get)
    ms = [r for r in step if r['Queue_Id'] + '/' + r['Stream_Id'] == main_q]
    gs = [(int(q['Start_Timestamp']) - int(p['End_Timestamp'])) / 1e3 for p, q in zip(ms, ms[1:])]
    import statistics as _st
    print(f"main-stream gaps: n={len(gs)} sum={sum(gs):.1f} us median={_st.median(gs):.2f} us "
          f"sum(<8us)={sum(g for g in gs if g < 8):.1f} us sum(>=8us)={sum(g for g in gs if g >= 8):.1f} us")
