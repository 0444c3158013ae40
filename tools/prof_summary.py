"""Per-step kernel time from a rocprofv3 --stats run of bench.py: python tools/prof_summary.py <dir> [steps] [top].
steps = 0 (default): the number of training steps the run executed, counted as embed_sort_kernel calls
(one per training forward)."""
import csv
import sys

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
if steps <= 0:
    steps = float(sum(int(r['Calls']) for r in rows if 'embed_sort_kernel' in r['Name']) or 1)
rows = [r for r in rows if 'spin_kernel' not in r['Name']]  # the bench's GPU-only section's spin kernel
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel ms {tot/1e6:.2f} over {steps:.0f} steps, per step {tot/1e6/steps:.3f}")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {int(r['Calls'])/steps:6.1f}/step avg "
          f"{float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:100]}")
