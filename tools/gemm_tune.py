"""Time every GEMM shape of one ERGM training step under each pipelined-kernel configuration.

Each (shape, config, split) is captured 20x into a HIP graph (torch.cuda.CUDAGraph) and replayed, so
host launch overhead is excluded; prints a table and the best config per shape, and writes
gpurun_out/gemm_tune.json.  Usage (on the GPU box):  python tools/gemm_tune.py [--quick] [--c5]
"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import _lib as L  # noqa: E402

T, E, F, LYR, VP = 2048, 768, 3072, 12, 50304
if "--c5" in sys.argv:  # config 5 geometry (GPT-2-medium, B=32, S=128); its forward GEMMs run fp8
    T, E, F, LYR = 4096, 1024, 4096, 24
if "--c4" in sys.argv:  # config 4 geometry (GPT-2-small, B=8, S=512)
    T = 4096
L2E = 2 * E * LYR
# --chain: the forward block GEMMs at the in-step row count (the forward runs as two batch-half chains)
TF = T // 2 if "--chain" in sys.argv else T
MK, KM, NK, KN = L.MK, L.KM, L.NK, L.KN
BF, FP = L.BF16, L.F32
# name, count/step, M, N, K, a_layout, lda, b_layout, ldb, epilogue, c_dtype
SHAPES = [
    ("fwd capkv", 1, T, L2E, E, MK, E + 8, KN, L2E, L.EPI_BIAS, BF),
    ("fwd c_attn", 12, TF, 3 * E, E, MK, E + 8, KN, 3 * E, L.EPI_BIAS, BF),
    ("fwd proj+resid", 24, TF, E, E, MK, E + 8, KN, E, L.EPI_BIAS_RESID, FP),
    ("fwd q_attn", 12, TF, E, E, MK, E + 8, KN, E, L.EPI_BIAS, BF),
    ("fwd c_fc+gelu", 12, TF, F, E, MK, E + 8, KN, F, L.EPI_BIAS_GELU, BF),
    ("fwd mlp proj+resid", 12, TF, E, F, MK, F + 8, KN, E, L.EPI_BIAS_RESID, FP),
    ("fwd lm_head", 1, T, VP, E, MK, E, NK, E, L.EPI_NONE, BF),
    ("bwd lm dX", 1, T, E, VP, MK, VP, KN, E, L.EPI_NONE, FP),
    ("bwd lm dW", 1, VP, E, T, KM, VP, KN, E, L.EPI_NONE, FP),
    ("bwd mproj dW", 12, F + 1, E, T, KM, F + 8, KN, E, L.EPI_NONE, FP),
    ("bwd dpre (gelu')", 12, T, F, E, MK, E, NK, E, L.EPI_GELU_BWD, BF),
    ("bwd fc dW", 12, E + 1, F, T, KM, E + 8, KN, F, L.EPI_NONE, FP),
    ("bwd fc dX", 12, T, E, F, MK, F, NK, F, L.EPI_NONE, FP),
    ("bwd ExE dW", 36, E + 1, E, T, KM, E + 8, KN, E, L.EPI_NONE, FP),
    ("bwd d_o", 24, T, E, E, MK, E, NK, E, L.EPI_NONE, BF),
    ("bwd q dX", 12, T, E, E, MK, E, NK, E, L.EPI_NONE, FP),
    ("bwd c_attn dW", 12, E + 1, 3 * E, T, KM, E + 8, KN, 3 * E, L.EPI_NONE, FP),
    ("bwd c_attn dX", 12, T, E, 3 * E, MK, 3 * E, NK, 3 * E, L.EPI_NONE, FP),
    ("bwd capkv dW", 1, E + 1, L2E, T, KM, E + 8, KN, L2E, L.EPI_NONE, FP),
    ("bwd dcap", 1, T, E, L2E, MK, L2E, NK, L2E, L.EPI_NONE, FP),
]
CFGS = [(64, 64), (128, 128), (128, 128), (128, 128), (256, 128), (128, 256), (256, 256), (128, 64), (64, 128),
        (256, 128), (128, 128), (64, 64), (128, 64), (64, 128), (128, 128), (128, 128),
        (64, 64), (64, 64), (128, 64), (64, 128), (128, 128), (128, 128),
        (256, 256), (128, 128), (128, 128),                       # 22-24 LDS-free epilogue variants
        (64, 64), (128, 128), (128, 128), (256, 256), (64, 128), (128, 128), (128, 128), (128, 128),  # 25-32 IL
        (64, 64), (64, 64), (64, 128), (128, 64), (128, 128),                                         # 33-37 KS2
        (64, 64), (128, 128), (128, 128), (128, 64), (64, 128), (128, 128), (256, 256), (64, 64), (128, 128)]  # 38-46
# 38-46: the v_mfma_f32_32x32x16_bf16 twins of cfgs 0, 2, 10, 7, 8, 15, 6, 11, 3
REPS = 20


def blas_compare():
    """torch.matmul (hipBLASLt) on the same shapes/transposes, bf16 in and out, vs ergm_gemm auto."""
    dev = torch.device("cuda:0")
    tot_b = tot_e = 0.0
    for (name, cnt, M, N, K, al, lda, bl, ldb, epi, cdt) in SHAPES:
        a = torch.randn(M, K, device=dev).bfloat16() if al == MK else torch.randn(K, M, device=dev).bfloat16().t()
        b = torch.randn(K, N, device=dev).bfloat16() if bl == KN else torch.randn(N, K, device=dev).bfloat16().t()
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            c = a @ b
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(REPS):
                torch.matmul(a, b, out=c)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        tb = e0.elapsed_time(e1) / (3 * REPS) * 1e3
        tot_b += tb * cnt
        print(f"{name:22s} x{cnt:2d} M={M:5d} N={N:5d} K={K:5d}  hipBLASLt {tb:8.1f}us "
              f"({2.0 * M * N * K / tb / 1e6:6.0f} TF)", flush=True)
    print(f"per-step GEMM time hipBLASLt (bf16 out, no epilogue): {tot_b / 1e3:.3f} ms")


def main():
    if "--blas" in sys.argv:
        return blas_compare()
    quick = "--quick" in sys.argv
    dev = torch.device("cuda:0")
    lib = L.load()
    g = torch.Generator(device="cpu").manual_seed(0)
    results = []
    total_best = 0.0
    total_auto = 0.0
    only_bwd = "--c5" in sys.argv
    only_dw = "--dw" in sys.argv
    for (name, cnt, M, N, K, al, lda, bl, ldb, epi, cdt) in SHAPES:
        if only_bwd and name.startswith("fwd") and name != "fwd lm_head":
            continue
        if only_dw and al != KM:
            continue
        if "--fwd" in sys.argv and not (name.startswith("fwd") and name not in ("fwd lm_head", "fwd capkv")):
            continue
        a_rows = M if al == MK else K
        b_rows = N if bl == NK else K
        A = (torch.randn(a_rows, lda, generator=g) * 0.1).bfloat16().to(dev)
        B = (torch.randn(b_rows, ldb, generator=g) * 0.1).bfloat16().to(dev)
        Cm = torch.zeros(M, N, dtype=torch.bfloat16 if cdt == BF else torch.float32, device=dev)
        bias = torch.randn(N + 8, device=dev)
        aux = None
        aux_out = None
        if epi == L.EPI_BIAS_RESID:
            aux = torch.randn(M, N, device=dev)
        if epi == L.EPI_GELU_BWD:
            aux = torch.randn(M, N, device=dev).bfloat16()
        if epi == L.EPI_BIAS_GELU:
            aux_out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        d = L.GemmDesc(M=M, N=N, K=K, lda=lda, ldb=ldb, ldc=N, a_layout=al, b_layout=bl, c_dtype=cdt,
                       epilogue=epi, alpha=1.0, bias=C.c_void_p(bias.data_ptr()),
                       aux=C.c_void_p(aux.data_ptr()) if aux is not None else None, ld_aux=N,
                       aux_out=C.c_void_p(aux_out.data_ptr()) if aux_out is not None else None, ld_aux_out=N,
                       split_k=0)
        flops = 2.0 * M * N * K
        row = {"name": name, "count": cnt, "M": M, "N": N, "K": K, "times": {}}

        def run_cfg(cfg, split):
            L.check(lib.ergm_gemm_tune(cfg, split), "tune")
            d.split_k = split if split > 1 else (1 if cfg >= 0 else 0)
            wsb = lib.ergm_gemm_workspace_size(C.byref(d))
            ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                L.check(lib.ergm_gemm(C.byref(d), C.c_void_p(A.data_ptr()), C.c_void_p(B.data_ptr()),
                                      C.c_void_p(Cm.data_ptr()), C.c_void_p(ws.data_ptr()), wsb,
                                      C.c_void_p(s.cuda_stream)), "gemm")
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s):
                for _ in range(REPS):
                    lib.ergm_gemm(C.byref(d), C.c_void_p(A.data_ptr()), C.c_void_p(B.data_ptr()),
                                  C.c_void_p(Cm.data_ptr()), C.c_void_p(ws.data_ptr()), wsb,
                                  C.c_void_p(torch.cuda.current_stream().cuda_stream))
            graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                graph.replay()
            e1.record()
            torch.cuda.synchronize()
            L.check(lib.ergm_gemm_tune(-1, 0), "tune")
            return e0.elapsed_time(e1) / (3 * REPS) * 1e3  # us

        row["times"]["auto"] = run_cfg(-1, 0)
        cfgs = range(len(CFGS)) if not quick else [0, 1, 3, 4, 7]
        if "--cfgs" in sys.argv:  # an explicit list, e.g. --cfgs 2,6,25,26
            cfgs = [int(c) for c in sys.argv[sys.argv.index("--cfgs") + 1].split(",")]
        if "--auto-only" in sys.argv:  # only the automatic plan of every shape (A/B of two builds)
            cfgs = []
        for cfg in cfgs:
            bm, bn = CFGS[cfg]
            tiles = -(-M // bm) * -(-N // bn)
            splits = [1]
            if tiles < 400 and "--nosplit" not in sys.argv:
                splits += [s for s in (2, 3, 4, 6, 8) if K // s >= 256 and tiles * s <= 2048]
            for sp in splits:
                try:
                    row["times"][f"c{cfg}s{sp}"] = run_cfg(cfg, sp)
                except Exception as ex:  # noqa: BLE001
                    row["times"][f"c{cfg}s{sp}"] = None
                    print("  fail", name, cfg, sp, ex, flush=True)
        valid = {k: v for k, v in row["times"].items() if v is not None and (k != "auto" or not cfgs)}
        best = min(valid, key=valid.get)
        row["best"] = best
        total_best += valid[best] * cnt
        total_auto += row["times"]["auto"] * cnt
        print(f"{name:22s} x{cnt:2d} M={M:5d} N={N:5d} K={K:5d}  auto {row['times']['auto']:8.1f}us "
              f"({flops / row['times']['auto'] / 1e6:6.0f} TF)  best {best:7s} {valid[best]:8.1f}us "
              f"({flops / valid[best] / 1e6:6.0f} TF)", flush=True)
        results.append(row)
    print(f"per-step GEMM time: auto {total_auto / 1e3:.3f} ms, best {total_best / 1e3:.3f} ms")
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/gemm_tune.json", "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
