"""Summary of tools/pmc_gemm.sh: per-dispatch mean of every counter over the GEMM dispatches of each pass."""
import csv
import glob
import sys
from collections import defaultdict

prefix, n = sys.argv[1], int(sys.argv[2])
for i in range(1, n + 1):
    files = glob.glob(f"{prefix}{i}/**/*counter_collection.csv", recursive=True)
    if not files:
        print("pass", i, "no counter file")
        continue
    acc, cnt = defaultdict(float), defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            if "gemm" not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(" ".join(f"{k}={acc[k] / max(1, len(cnt[k])):.4g}" for k in sorted(acc)))
