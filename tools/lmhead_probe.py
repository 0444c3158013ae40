"""Split the LM-head GEMM's time into a K-proportional main loop and a fixed part (prologue, epilogue
stores, tail): time [M, K] x [K, N] (MK x NK, bf16 out, the tied-head layout) for several K, HIP-graph
replayed.  Usage: python tools/lmhead_probe.py [cfg [M N [--small]]]"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import _lib as L  # noqa: E402


def time_gemm(lib, M, N, K, cfg, out_dtype=torch.bfloat16, reps=20):
    dev = torch.device("cuda:0")
    A = (torch.randn(M, K, device=dev) * 0.1).bfloat16()
    B = (torch.randn(N, K, device=dev) * 0.1).bfloat16()
    Cm = torch.empty(M, N, dtype=out_dtype, device=dev)
    d = L.GemmDesc(M=M, N=N, K=K, lda=K, ldb=K, ldc=N, a_layout=L.MK, b_layout=L.NK,
                   c_dtype=L.BF16 if out_dtype == torch.bfloat16 else L.F32, epilogue=L.EPI_NONE, alpha=1.0,
                   split_k=1 if cfg >= 0 else 0)
    L.check(lib.ergm_gemm_tune(cfg, 1 if cfg >= 0 else 0), "tune")
    s = torch.cuda.Stream(dev)
    args = (C.byref(d), C.c_void_p(A.data_ptr()), C.c_void_p(B.data_ptr()), C.c_void_p(Cm.data_ptr()), None, 0)
    with torch.cuda.stream(s):
        L.check(lib.ergm_gemm(*args, C.c_void_p(s.cuda_stream)), "gemm")
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            lib.ergm_gemm(*args, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    L.check(lib.ergm_gemm_tune(-1, 0), "tune")
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def main():
    lib = L.load()
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    M, N = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (2048, 50304)
    if "--small" in sys.argv:  # fixed vs K-proportional cost of a small activation GEMM
        for K in (64, 128, 256, 768, 1536):
            t = time_gemm(lib, M, N, K, cfg)
            print(f"M={M} N={N} K={K}: {t:8.2f} us  {2.0 * M * N * K / t / 1e6:7.0f} TF", flush=True)
        return
    ts = {}
    for K in (768, 1536, 3072):
        ts[K] = time_gemm(lib, M, N, K, cfg)
        print(f"M={M} N={N} K={K}: {ts[K]:8.1f} us  {2.0 * M * N * K / ts[K] / 1e6:7.0f} TF", flush=True)
    per_k = (ts[3072] - ts[768]) / (3072 - 768)
    print(f"main loop {per_k * 768:.1f} us per 768 of K ({2.0 * M * N / per_k / 1e6:.0f} TF in the loop), "
          f"fixed part {ts[768] - per_k * 768:.1f} us")
    tf = time_gemm(lib, M, N, 768, cfg, torch.float32)
    print(f"f32 output at K=768: {tf:.1f} us (store bytes x2)")


if __name__ == "__main__":
    main()
