"""HBM bytes per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of bench.py.

Run on the GPU box (each counter in its own pass, kernel-trace only, no other tracing):
    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py ...
then:  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_traffic.json

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, "HBM"): rocprofv3 reports FETCH_SIZE / WRITE_SIZE in
KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of wide coalesced streaming reads, so it is
doubled.  The AdamW kernel (30 B/param of pure streaming: 16 B read + 14 B written) is reported beside
the GEMM as the calibration of both corrections.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)  # kernel name -> [value per dispatch]
    for f in files:
        acc = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (f, r["Dispatch_Id"])
            acc[key] += float(r["Counter_Value"])   # summed over dimensions (XCD/channel) if split
            names[key] = r["Kernel_Name"]
        for key, v in acc.items():
            per[names[key]].append(v * 1024.0)      # KiB -> bytes
    return per


def main():
    fdir, wdir, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = _load(fdir, "FETCH_SIZE")
    write = _load(wdir, "WRITE_SIZE")
    from ergm_amd.config import gpt2_small
    from ergm_amd.params import build_layout
    cfg = gpt2_small()
    T, E, Vp = 16 * 128, cfg.n_embd, 50304
    n_flat = build_layout(cfg.vocab_size, cfg.n_embd, cfg.n_layer, cfg.inner, cfg.n_positions).total

    def pick(pred):
        ks = [k for k in fetch if pred(k)]
        if not ks:
            return None
        k = ks[0]
        fb = 2.0 * statistics.median(fetch[k])
        wb = statistics.median(write.get(k, [0.0]))
        return k, fb, wb

    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of bench.py; "
                     "FETCH_SIZE doubled (gfx950 streaming-read correction), KiB -> bytes; median over dispatches"}
    lm = pick(lambda k: "gemm_pipe_kernel<256, 256, 4, 2, 2, false, false, 0, true" in k)
    if lm:
        k, fb, wb = lm
        from bench import lmhead_split_cols
        n0 = lmhead_split_cols(T, Vp)  # the main launch's columns (the bench's roofline kernel)
        alg = 2 * T * E + 2 * n0 * E + 2 * T * n0   # A [T,E] + wte [n0,E] bf16 read, logits [T,n0] bf16 written
        res["lm_head_fwd"] = {"kernel": k, "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                              "algorithmic_bytes": alg, "ratio": (fb + wb) / alg}
    # the weight-gradient GEMM class (bench.py's roofline): every KM x KN pipelined GEMM dispatch; mean
    # bytes per launch over the class against the mean algorithmic bytes of its C2 launches
    dwk = [k for k in fetch if (("gemm_pipe_kernel<" in k or "gemm_ws_kernel<" in k) and ", true, true, " in k) or "gemm_dw2_kernel<" in k]
    if dwk:
        F, L = 4 * E, cfg.n_layer
        shapes = [(Vp, E)] + [(F + 1, E), (E + 1, F), (E + 1, E), (E + 1, E), (E + 1, E), (E + 1, 3 * E)] * L + \
                 [(E + 1, 2 * E * L)]
        nd = sum(len(fetch[k]) for k in dwk)
        # per launch: the class's algorithmic bytes per step over its launches per step (74 single launches,
        # or fewer when pairs of them run as one grouped launch); steps = training forwards in the pass
        steps = sum(len(v) for k, v in fetch.items() if "embed_sort_kernel" in k) or 1
        alg = sum(2 * T * m + 2 * T * n + 4 * m * n for m, n in shapes) / (nd / steps)
        fb = 2.0 * sum(sum(fetch[k]) for k in dwk) / nd
        wb = sum(sum(write.get(k, [])) for k in dwk) / max(1, sum(len(write.get(k, [])) for k in dwk))
        res["dw_class"] = {"kernels": [k.split("(")[0] for k in dwk], "dispatches": nd, "fetch_bytes": fb,
                           "write_bytes": wb, "hbm_bytes": fb + wb, "algorithmic_bytes": alg,
                           "ratio": (fb + wb) / alg,
                           "launches_per_step": nd / steps,
                           "note": "mean per launch over the class; algorithmic = X^T and dY bf16 read once + dW f32 "
                                   "written once, summed over the step's 74 GEMMs / the class's launches per step"}
    ad = pick(lambda k: "adamw_kernel" in k)
    if ad:
        k, fb, wb = ad
        res["adamw_calibration"] = {"kernel": k, "n_params": n_flat, "fetch_bytes": fb, "write_bytes": wb,
                                    "expected_read": 16 * n_flat, "expected_write": 14 * n_flat,
                                    "read_ratio": fb / (16 * n_flat), "write_ratio": wb / (14 * n_flat)}
    allk = {}
    for k in fetch:
        allk[k.split("(")[0][:90]] = {"fetch_bytes": 2.0 * statistics.median(fetch[k]),
                                      "write_bytes": statistics.median(write.get(k, [0.0])),
                                      "dispatches": len(fetch[k])}
    res["per_kernel_median"] = allk
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel_median"}, indent=1))


if __name__ == "__main__":
    main()
