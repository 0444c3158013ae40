"""Capture single library ops in a torch CUDA graph (bisecting the whole-step capture crash, round 6).
Usage (GPU box): python tools/capture_ops.py <op>   op: ln | gemm | gemm_big (the 256x256 LM-head tile, 128 KB LDS)"""
import faulthandler
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    faulthandler.enable()
    from ergm_amd import _lib as L
    from ergm_amd import ops
    op = sys.argv[1]
    dev = torch.device("cuda:0")
    if op == "ln":
        x = torch.randn(2048, 768, device=dev)
        w, b = torch.ones(768, device=dev), torch.zeros(768, device=dev)
        run = lambda: ops.layernorm_fwd(x, w, b)  # noqa: E731
    else:
        M, N, K = (2048, 50304, 768) if op == "gemm_big" else (1024, 1024, 1024)
        a = torch.randn(M, K, device=dev).bfloat16()
        bt = torch.randn(N, K, device=dev).bfloat16()
        c = torch.empty(M, N, device=dev)
        run = lambda: ops.gemm(a, bt, M, N, K, L.MK, L.NK, out=c)  # noqa: E731
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        ref = run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    print(f"{op}: capturing", flush=True)
    with torch.cuda.graph(g, stream=s):
        out = run()
    print(f"{op}: captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    r0 = ref[0] if isinstance(ref, tuple) else ref
    o0 = out[0] if isinstance(out, tuple) else out
    print(f"{op}: replay matches eager: {torch.equal(r0, o0)}", flush=True)


if __name__ == "__main__":
    main()
