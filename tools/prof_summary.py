import csv, sys
d = sys.argv[1]; steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel ms {tot/1e6:.2f}  per step {tot/1e6/steps:.3f}")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {int(r['Calls'])/steps:6.1f}/step avg {float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:100]}")
