"""Do two independent launch chains on two HIP streams overlap on MI355X?  Times 2N launches of one GEMM shape on
one stream against N on each of two streams (no tracer), for the forward's shapes (M = 1024 per batch-half chain).
Prints us per launch for both and their ratio (1.0 = no overlap, 0.5 = perfect overlap)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ergm_amd import _lib as L, ops  # noqa: E402


def run(shape, n=200):
    M, N, K = shape
    dev = torch.device("cuda:0")
    A = [torch.randn(M, K, device=dev).bfloat16() for _ in range(2)]
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    W = (0.05 * torch.randn(K, N, device=dev)).bfloat16()
    C = [torch.empty(M, N, device=dev) for _ in range(2)]
    s = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    import ctypes as Cc
    lib = L.load()
    descs = [L.GemmDesc(M=M, N=N, K=K, lda=K, ldb=N, ldc=N, a_layout=L.MK, b_layout=L.KN, c_dtype=L.F32,
                        epilogue=L.EPI_NONE, alpha=1.0, split_k=1) for _ in range(2)]
    args = [(Cc.byref(descs[k]), Cc.c_void_p(A[k].data_ptr()), Cc.c_void_p(W.data_ptr()), Cc.c_void_p(C[k].data_ptr()),
             Cc.c_void_p(ws.data_ptr()), ws.numel(), Cc.c_void_p(s[k].cuda_stream)) for k in range(2)]

    def chain(k, cnt):
        for _ in range(cnt):
            lib.ergm_gemm(*args[k])
    for _ in range(3):  # warm-up
        chain(0, 20)
        chain(1, 20)
    torch.cuda.synchronize()
    res = {}
    for mode in ("one", "two", "one", "two"):
        torch.cuda.synchronize()
        # the whole chain is enqueued behind a spin kernel, then timed on the device: no host in the loop
        torch.cuda._sleep(int(2.4e9 * 0.03))
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(2):
            s[k].wait_event(e0)
        if mode == "one":
            chain(0, 2 * n)
        else:
            for i in range(n):  # interleaved enqueue, like the executor's two forward chains
                chain(0, 1)
                chain(1, 1)
        e1 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for k in range(2):
            e1[k].record(s[k])
        torch.cuda.synchronize()
        res[mode] = max(e0.elapsed_time(e) for e in e1) * 1e3 / (2 * n)
    print(f"M={M} N={N} K={K}: one stream {res['one']:.2f} us/launch, two streams {res['two']:.2f} us/launch, "
          f"ratio {res['two'] / res['one']:.2f}", flush=True)


if __name__ == "__main__":
    for shape in ((1024, 768, 768), (1024, 2304, 768), (1024, 3072, 768), (1024, 768, 3072), (2048, 768, 768)):
        run(shape)
