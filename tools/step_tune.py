"""Tune GEMM configurations inside the running training step.

Isolated GEMM timings (tools/gemm_tune.py) do not predict the step: its kernels share the CUs across
four streams (profiles/r01_overlap_experiments.txt).  This tool runs the real bench.py step, records
the distinct GEMM shapes (ergm_gemm_trace), and for each shape — largest first — tries candidate
configurations through ergm_gemm_set_override, keeping one only if the measured step time drops by
more than the noise threshold (and again on a confirming re-measurement).

    python tools/step_tune.py [--config c2|c4|c5] [--steps 30] [--splits 1,2,4] [--out gpurun_out/step_tune.json]
    python tools/step_tune.py --config c5 --f8      # the fp8 / MX GEMMs' tiles (ergm_gemm_f8_set_override)

Split-K candidates (--splits) use the plan's scratch for their slab; a split that does not fit is
reported by the GEMM as an error and skipped.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ergm_amd import _lib as L  # noqa: E402

CANDIDATES = [0, 2, 10, 14, 15, 6, 4, 9, 1, 3, 7, 8, 11, 12, 13, 22, 23, 24,
              38, 39, 40, 41, 42, 43, 44, 45, 46]  # kCfgs indices (gemm.hip); 38-46: v_mfma_f32_32x32x16_bf16
F8_TILE = {0: (128, 128), 1: (256, 128), 2: (128, 128), 3: (256, 256), 4: (64, 64)}  # kF8Cfgs (gemm.hip)
TILE = {0: (64, 64), 1: (128, 128), 2: (128, 128), 3: (128, 128), 4: (256, 128), 6: (256, 256), 7: (128, 64),
        8: (64, 128), 9: (256, 128), 10: (128, 128), 11: (64, 64), 12: (128, 64), 13: (64, 128), 14: (128, 128),
        15: (128, 128), 16: (64, 64), 17: (64, 64), 18: (128, 64), 19: (64, 128), 20: (128, 128), 21: (128, 128),
        22: (256, 256), 23: (128, 128), 24: (128, 128), 25: (64, 64), 26: (128, 128), 27: (128, 128),
        28: (256, 256), 29: (64, 128), 30: (128, 128), 31: (128, 128), 32: (128, 128), 33: (64, 64), 34: (64, 64),
        35: (64, 128), 36: (128, 64), 37: (128, 128), 38: (64, 64), 39: (128, 128), 40: (128, 128), 41: (128, 64),
        42: (64, 128), 43: (128, 128), 44: (256, 256), 45: (64, 64), 46: (128, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--threshold", type=float, default=0.005)
    ap.add_argument("--max-shapes", type=int, default=24)
    ap.add_argument("--splits", default="1")
    ap.add_argument("--out", default="gpurun_out/step_tune.json")
    ap.add_argument("--candidates", default=None, help="comma-separated kCfgs indices (default: the built-in list)")
    ap.add_argument("--f8", action="store_true", help="tune the fp8 / MX GEMMs (traced with a_layout 16) instead")
    ap.add_argument("--shapes", default=None, help="comma-separated MxNxK shapes to tune (default: every traced shape)")
    args = ap.parse_args()
    from ergm_amd.config import ERGMConfig
    from ergm_amd.data import synthetic_batch
    from ergm_amd.model import GPT2LMHeadModel
    from ergm_amd.optim import FusedAdamW

    dev = torch.device("cuda:0")
    mname, S, turns, B, Fd, fp8, _ = bench.CONFIGS[args.config]
    cfg = ERGMConfig(**bench.MODELS[mname], feat_dim=Fd, fp8=fp8)
    model = GPT2LMHeadModel(cfg, device=dev)
    model.init_weights(seed=0)
    opt = FusedAdamW([model.flat], lr=2e-5, model=model, overlap=True)
    batch = synthetic_batch(B, S, n_turns=turns, seed=1000, feat_dim=Fd)
    kw = dict(input_ids=batch["input_ids"], token_type_ids=batch["token_type_ids"], labels=batch["labels"],
              emotion_labels=batch["emotion_labels"], caption_ids=batch["caption_ids"], imgs=batch["visual_feat"],
              auds=batch["audio_feat"])
    kw = {k: v.to(dev) for k, v in kw.items()}
    lib = L.load()

    def step():
        out = model(**kw)
        opt.zero_grad()
        out.loss.backward()
        opt.step()

    def measure(steps=args.steps):
        for _ in range(2):  # let the previous configuration's work drain
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return 1000.0 * (time.perf_counter() - t0) / steps

    def set_cfg(key, cfg_split):
        M, N, K, al, bl = key
        c, sp = cfg_split if cfg_split is not None else (-1, 1)
        if al == 16:  # an fp8 / MX GEMM
            L.check(lib.ergm_gemm_f8_set_override(M, N, K, c), "f8 override")
        else:
            L.check(lib.ergm_gemm_set_override(M, N, K, al, bl, c, sp), "override")

    def ab(key, inc, cand, rounds=2):
        """Interleaved A/B/A/B step times of the incumbent and the candidate configuration."""
        a = b = 0.0
        for _ in range(rounds):
            set_cfg(key, inc)
            a += measure()
            set_cfg(key, cand)
            b += measure()
        set_cfg(key, inc)
        return a / rounds, b / rounds

    lib.ergm_gemm_trace(1, None, 0)
    step()
    torch.cuda.synchronize()
    buf = (C.c_int * (256 * 5))()
    n = lib.ergm_gemm_trace(0, buf, 256)
    shapes = [tuple(buf[i * 5:(i + 1) * 5]) for i in range(n)]
    shapes = [t for t in shapes if (t[3] == 16) == args.f8]
    shapes.sort(key=lambda t: -2.0 * t[0] * t[1] * t[2])
    if args.shapes:
        want = {tuple(int(x) for x in w.split("x")) for w in args.shapes.split(",")}
        shapes = [t for t in shapes if t[:3] in want]
    shapes = shapes[:args.max_shapes]
    for _ in range(10):
        step()
    base = measure(3 * args.steps)
    print(f"{len(shapes)} GEMM shapes; baseline {base:.3f} ms/step", flush=True)
    chosen = {}
    for key in shapes:
        M, N, K, al, bl = key
        best = None  # None = the automatic choice
        splits = [int(x) for x in args.splits.split(",")]
        if args.f8:
            splits = [1]
        cands = [int(x) for x in args.candidates.split(",")] if args.candidates else \
            (list(F8_TILE) if args.f8 else CANDIDATES)
        for c, sp in [(c, sp) for sp in splits for c in cands]:
            bm, bn = (F8_TILE if args.f8 else TILE)[c]
            tiles = -(-M // bm) * -(-N // bn)
            if tiles < 24 or tiles > 20000 or (sp > 1 and (K // sp < 512 or tiles * sp > 2048)):
                continue
            try:
                t_inc, t_cand = ab(key, best, (c, sp), rounds=1)
                if t_cand < t_inc * (1.0 - args.threshold):
                    t_inc, t_cand = ab(key, best, (c, sp), rounds=2)  # confirm
                    if t_cand < t_inc * (1.0 - args.threshold):
                        print(f"  {M}x{N}x{K} al{al} bl{bl}: c{c}s{sp} {t_cand:.3f} vs {t_inc:.3f} ms/step", flush=True)
                        best = (c, sp)
                        set_cfg(key, best)
            except Exception as ex:  # noqa: BLE001  (a configuration the shape cannot take)
                print(f"  {M}x{N}x{K} c{c}s{sp}: {ex}", flush=True)
                set_cfg(key, best)
        if best is not None:
            chosen[key] = best
        print(f"shape {M}x{N}x{K} al{al} bl{bl}: {'c%ds%d' % best if best else 'auto'}", flush=True)
    # final A/B of the whole table against the automatic choice
    t_new = t_old = 0.0
    for _ in range(3):
        t_new += measure(2 * args.steps)
        for key in chosen:
            set_cfg(key, None)
        t_old += measure(2 * args.steps)
        for key, v in chosen.items():
            set_cfg(key, v)
    base, final = t_old / 3, t_new / 3
    print(f"final {final:.3f} ms/step vs automatic {base:.3f} ({100 * (1 - final / base):.1f} % faster)", flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"config": args.config, "baseline_ms": base, "final_ms": final,
                   "overrides": [list(k) + list(v) for k, v in chosen.items()]}, f, indent=1)


if __name__ == "__main__":
    main()
