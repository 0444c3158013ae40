"""Per-K-step cost of the pipelined GEMM configurations: one tile per CU (256 tiles), K swept, the
slope of time vs K = the steady-state cost of one 64-deep K step of one workgroup.
Usage (GPU box): python tools/gemm_kslope.py"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import _lib as L  # noqa: E402

CFGS = {0: (64, 64), 2: (128, 128), 6: (256, 256), 10: (128, 128), 16: (64, 64), 17: (64, 64), 18: (128, 64),
        19: (64, 128), 20: (128, 128), 21: (128, 128)}


def main():
    dev = torch.device("cuda:0")
    lib = L.load()
    per_cu = int(sys.argv[1]) if len(sys.argv) > 1 else 1   # tiles per CU (256 CUs)
    for cfg, (bm, bn) in CFGS.items():
        for al, bl, tag in ((L.MK, L.NK, "MKxNK"), (L.KM, L.KN, "KMxKN")):
            M, N = bm * 16 * per_cu, bn * 16
            pts = []
            for K in (512, 1024, 2048, 4096):
                A = torch.randn(M * K, device=dev).bfloat16()
                B = torch.randn(N * K, device=dev).bfloat16()
                Cm = torch.empty(M, N, dtype=torch.float32, device=dev)
                d = L.GemmDesc(M=M, N=N, K=K, lda=K if al == L.MK else M, ldb=K if bl == L.NK else N, ldc=N,
                               a_layout=al, b_layout=bl, c_dtype=L.F32, epilogue=L.EPI_NONE, alpha=1.0,
                               split_k=1)
                L.check(lib.ergm_gemm_tune(cfg, 1), "tune")
                s = torch.cuda.current_stream().cuda_stream

                def run():
                    L.check(lib.ergm_gemm(C.byref(d), C.c_void_p(A.data_ptr()), C.c_void_p(B.data_ptr()),
                                          C.c_void_p(Cm.data_ptr()), None, 0, C.c_void_p(s)), "gemm")
                run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    run()
                e1.record()
                torch.cuda.synchronize()
                pts.append((K, e0.elapsed_time(e1) / 50 * 1e3))
            L.check(lib.ergm_gemm_tune(-1, 0), "tune")
            (k0, t0), (k1, t1) = pts[1], pts[-1]
            slope = (t1 - t0) / ((k1 - k0) / 64)  # us per K step
            cyc = slope * 1e-6 * 2.4e9
            mfma_cyc = per_cu * bm * bn * 64 * 2 / (2.5e15 / 256 / 2.4e9)  # ideal cycles at per-CU peak
            fill = per_cu * (bm + bn) * 64 * 2 / (slope * 1e-6) / 1e9
            print(f"cfg{cfg:<2d} {bm}x{bn} {tag}: " + " ".join(f"K={k}:{t:.1f}us" for k, t in pts) +
                  f" | step {slope * 1e3:.0f} ns = {cyc:.0f} cyc (MFMA ideal {mfma_cyc:.0f}), fill {fill:.0f} GB/s/CU",
                  flush=True)


if __name__ == "__main__":
    main()
