"""Run one GEMM configuration repeatedly (for rocprofv3 PMC passes on a single kernel).
Usage: python tools/gemm_one.py CFG LAYOUT M N K REPS   (LAYOUT: MKxNK | KMxKN | MKxKN)"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import _lib as L  # noqa: E402


def main():
    cfg, lay = int(sys.argv[1]), sys.argv[2]
    M, N, K, reps = (int(x) for x in sys.argv[3:7])
    al = L.MK if lay.startswith("MK") else L.KM
    bl = L.NK if lay.endswith("NK") else L.KN
    dev = torch.device("cuda:0")
    lib = L.load()
    A = torch.randn(M * K, device=dev).bfloat16()
    B = torch.randn(N * K, device=dev).bfloat16()
    Cm = torch.empty(M, N, dtype=torch.float32, device=dev)
    d = L.GemmDesc(M=M, N=N, K=K, lda=K if al == L.MK else M, ldb=K if bl == L.NK else N, ldc=N, a_layout=al,
                   b_layout=bl, c_dtype=L.F32, epilogue=L.EPI_NONE, alpha=1.0, split_k=1)
    L.check(lib.ergm_gemm_tune(cfg, 1), "tune")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(reps):
        L.check(lib.ergm_gemm(C.byref(d), C.c_void_p(A.data_ptr()), C.c_void_p(B.data_ptr()),
                              C.c_void_p(Cm.data_ptr()), None, 0, s), "gemm")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
