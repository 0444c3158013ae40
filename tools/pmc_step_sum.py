"""Per kernel-class sums of tools/pmc_step.sh's counters (all dispatches of each class over the run)."""
import csv
import glob
import sys
from collections import defaultdict


def cls(name):
    n = name.split("(")[0]
    if "gemm_dw2" in n or ("gemm_pipe_kernel<" in n and ", true, true, " in n):
        return "gemm dW"
    if "gemm" in n or "splitk" in n:
        return "gemm other"
    for k in ("adamw", "ln_", "attn", "xent", "embed", "dropout"):
        if k in n:
            return k.strip("_")
    return "other"


prefix, n = sys.argv[1], int(sys.argv[2])
tot = defaultdict(lambda: defaultdict(float))
for i in range(1, n + 1):
    for f in glob.glob(f"{prefix}{i}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            tot[cls(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
for c, d in sorted(tot.items()):
    print(f"{c:12s} " + " ".join(f"{k}={v:.4g}" for k, v in sorted(d.items())))
    w = d.get("SQ_WAVE_CYCLES", 0)
    if w:
        print(f"{'':12s} wait {d.get('SQ_WAIT_ANY', 0) / w:.2f}  issue-stall {d.get('SQ_WAIT_INST_ANY', 0) / w:.2f}  "
              f"active {d.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}", end="")
    g = d.get("GRBM_GUI_ACTIVE", 0)
    if g:
        print(f"  TA busy {d.get('TA_TA_BUSY', 0) / (g / 8 * 256):.2f}", end="")
    h, m = d.get("TCC_HIT_sum", 0), d.get("TCC_MISS_sum", 0)
    if h + m:
        print(f"  L2 hit {h / (h + m):.2f}", end="")
    print()
