"""Isolated timing (HIP graph, 20 launches per replay) of the fused c_attn + causal attention kernel
against the separate GEMM + attention launches, at the C2 batch (B=16) and one forward chain (B=8).
Usage: python tools/qkv_attn_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import _lib as L  # noqa: E402
from ergm_amd import ops  # noqa: E402


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3


def main():
    dev = torch.device("cuda:0")
    H, S, E = 12, 128, 768
    for B in (16, 8):
        x = (torch.randn(B * S, E + 8, device=dev) * 0.5).bfloat16()[:, :E]
        w = (torch.randn(E, 3 * E, device=dev) * E ** -0.5).bfloat16()
        bias = torch.randn(3 * E, device=dev) * 0.1
        qkv = torch.empty(B * S, 3 * E, dtype=torch.bfloat16, device=dev)
        o = torch.empty(B * S, E, dtype=torch.bfloat16, device=dev)
        lse = torch.empty(B, H, S, device=dev)
        t_f = timed(lambda: ops.qkv_attn_fwd(x, w, bias, B, H, S, qkv, o, lse))
        t_g = timed(lambda: ops.gemm(x, w, B * S, 3 * E, E, L.MK, L.KN, out=qkv, epilogue=L.EPI_BIAS, bias=bias))
        t_a = timed(lambda: ops.attn_fwd(qkv[:, :E], qkv[:, E:2 * E], qkv[:, 2 * E:], B, H, S, S, True, o, lse))
        print(f"B={B}: fused {t_f:6.2f} us   separate GEMM {t_g:6.2f} + attention {t_a:6.2f} = {t_g + t_a:6.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
