"""Isolated timing of the non-GEMM kernels at the training step's shapes (C2: T = 16 x 128 tokens,
GPT-2-small), each captured 20x into a HIP graph and replayed (no launch overhead, no concurrency).
Prints time and effective HBM rate against the algorithmic bytes.  Usage (GPU box):
python tools/op_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import _lib as L  # noqa: E402
from ergm_amd import ops  # noqa: E402

REPS = 20
B, S, E, H, V, VP = 16, 128, 768, 12, 50260, 50304
T = B * S


def timed(fn):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(REPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * REPS) * 1e3


def report(name, us, nbytes):
    print(f"{name:34s} {us:8.2f} us   {nbytes / 1e6:8.1f} MB   {nbytes / us / 1e3:7.0f} GB/s", flush=True)


def main():
    dev = torch.device("cuda:0")
    lib = L.load()
    x = torch.randn(T, E, device=dev)
    gam, bet = torch.rand(E, device=dev) + 0.5, torch.randn(E, device=dev)
    y, mean, rstd = ops.layernorm_fwd(x, gam, bet)
    report("layernorm_fwd", timed(lambda: ops.layernorm_fwd(x, gam, bet)), T * E * 4 + T * E * 2 + T * 8)
    dy = torch.randn(T, E, device=dev)
    dres = torch.zeros(T, E, device=dev)
    report("layernorm_bwd (main+reduce)", timed(lambda: ops.layernorm_bwd(dy, x, mean, rstd, gam, dres)),
           T * E * (4 + 4 + 8 + 2))
    for causal, Sk in ((True, S), (False, S)):
        qkv = torch.randn(T, 3 * E, device=dev).bfloat16()
        q, k, v = qkv[:, :E], qkv[:, E:2 * E], qkv[:, 2 * E:]
        o, lse = ops.attn_fwd(q, k, v, B, H, S, Sk, causal)
        tag = "causal" if causal else "cross"
        report(f"attn_fwd {tag}", timed(lambda: ops.attn_fwd(q, k, v, B, H, S, Sk, causal)), 4 * T * E * 2)
        do = torch.randn(T, E, device=dev).bfloat16()
        report(f"attn_bwd {tag}", timed(lambda: ops.attn_bwd(q, k, v, o, do, lse, B, H, S, Sk, causal)), 8 * T * E * 2)
    logits = torch.randn(T, VP, device=dev).bfloat16()
    labels = torch.randint(0, V, (B, S), device=dev)
    nv = torch.full((4,), T, dtype=torch.int32, device=dev)
    report("xent fwd+bwd", timed(lambda: ops.xent(logits, labels, nv, V)), 2 * T * VP * 2)
    n = 152_848_128
    p, g, m, vv = (torch.randn(n, device=dev) for _ in range(4))
    pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
    report("adamw (whole model)", timed(lambda: ops.adamw_step(p, g, m, vv, pb, 1e-4, 0.9, 0.999, 1e-8, 0.01, 3)),
           30 * n)


if __name__ == "__main__":
    main()
