"""MFMA utilisation from one rocprofv3 PMC pass of bench.py (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE,
SQ_INSTS_VALU_MFMA_MOPS_BF16 — 2 SQ + 1 GRBM counters, within one pass's limits):

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 \\
        -d gpurun_out/pmc_mfma -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 ...
    python tools/pmc_mfma.py gpurun_out/pmc_mfma [out.json]

Per dispatch: MFMA busy % = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (GUI cycles x SIMDs) (the MFMA_UTIL expression
of rocprofiler-sdk's counter_defs.yaml for gfx950), with GUI cycles = GRBM_GUI_ACTIVE / 8: rocprofv3
reports the sum over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back); counted bf16 FLOPs = MOPS_BF16 x
512, set against the kernel's algorithmic FLOPs where known (the LM-head GEMM: 2·T·Vp·E).  Kernels on
concurrent streams overlap, so per-kernel busy % is over each kernel's own active cycles.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

SIMDS = 256 * 4


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = defaultdict(lambda: {"busy": 0.0, "gui": 0.0, "mops": 0.0, "name": ""})
    for f in files:
        for r in csv.DictReader(open(f)):
            key = (f, r["Dispatch_Id"])
            e = disp[key]
            e["name"] = r["Kernel_Name"]
            v = float(r["Counter_Value"])
            c = r["Counter_Name"]
            if c == "SQ_VALU_MFMA_BUSY_CYCLES":
                e["busy"] += v
            elif c == "GRBM_GUI_ACTIVE":
                e["gui"] = max(e["gui"], v / 8.0)  # reported as the sum over the 8 XCDs
            elif c == "SQ_INSTS_VALU_MFMA_MOPS_BF16":
                e["mops"] += v
    return list(disp.values())


def main():
    d = sys.argv[1]
    rows = load(d)
    per = defaultdict(list)
    for e in rows:
        per[e["name"]].append(e)
    out = {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 "
                     "(one pass) of bench.py; busy % = busy / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)", "kernels": {}}
    tot_busy = tot_gui = 0.0
    for name, es in per.items():
        busy = statistics.median(e["busy"] for e in es)
        gui = statistics.median(e["gui"] for e in es)
        mops = statistics.median(e["mops"] for e in es)
        tot_busy += sum(e["busy"] for e in es)
        tot_gui += sum(e["gui"] for e in es)
        if gui > 0:
            out["kernels"][name[:110]] = {"dispatches": len(es), "mfma_busy_pct": round(100 * busy / (gui * SIMDS), 2),
                                          "bf16_flops_counted": mops * 512}
    lm = [k for k in out["kernels"] if "gemm_pipe_kernel<256, 256, 4, 2, 2, false, false, 0, true" in k]
    if lm:
        rec = out["kernels"][lm[0]]
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import lmhead_split_cols
        alg = 2.0 * 2048 * lmhead_split_cols(2048, 50304) * 768  # the main launch (bench's roofline kernel)
        out["lm_head_fwd"] = dict(rec, algorithmic_flops=alg, counted_over_algorithmic=rec["bf16_flops_counted"] / alg)
    dw = [e for e in rows if ((("gemm_pipe_kernel<" in e["name"] or "gemm_ws_kernel<" in e["name"]) and ", true, true, " in e["name"]) or
                              "gemm_dw2_kernel<" in e["name"]) and e["gui"] > 0]  # single and grouped launches
    if dw:
        out["dw_class"] = {"dispatches": len(dw),
                           "mfma_busy_pct": round(100 * sum(e["busy"] for e in dw) / (sum(e["gui"] for e in dw) * SIMDS), 2),
                           "bf16_flops_counted_per_launch": sum(e["mops"] for e in dw) * 512 / len(dw)}
        print("dW class:", out["dw_class"])
    top = sorted(out["kernels"].items(), key=lambda kv: -kv[1]["mfma_busy_pct"])[:12]
    for k, v in top:
        print(f"{v['mfma_busy_pct']:6.2f}%  x{v['dispatches']:4d}  {k}")
    print("LM head:", out.get("lm_head_fwd"))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
