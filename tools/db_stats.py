"""Per-kernel totals from a rocprofv3 rocpd database (run_results.db): python tools/db_stats.py DB STEPS [TOP]."""
import collections
import sqlite3
import sys

db, steps = sys.argv[1], float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
c = sqlite3.connect(db)
agg = collections.defaultdict(lambda: [0, 0.0])
for n, d, gx, gy, wx in c.execute("select name, duration, grid_x, grid_y, workgroup_x from kernels"):
    k = f"{n.split('(')[0][:90]} g={gx // max(wx, 1)}x{gy}"
    agg[k][0] += 1
    agg[k][1] += d / 1e3
tot = sum(v[1] for v in agg.values())
print(f"total kernel time {tot / steps:.1f} us per step")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"  {v[1] / steps:9.1f} us/step  n/step={v[0] / steps:5.1f}  avg={v[1] / v[0]:7.1f}  {k}")
